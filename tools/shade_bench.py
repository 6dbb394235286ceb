"""Shading-kernel throughput on one GPU: simple::kernel, whitted::kernel
and multi_hit<16> at 1080p on hf1M, rays/s from the device counters over K timed frames, for each
waves-per-SIMD register budget.  Prints one JSON line per (kernel, occ).

    python tools/shade_bench.py [--scene hf1M] [--frames 10] [--frames-per-launch F]

--frames-per-launch F > 1: the frames run as frames/F persistent launches of F frames each
(vrh_render_batch, frames in flight, as hip_sched::frames) instead of one hip_sched::frame each.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="hf1M")
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--occ", default="0,1,6,8")
    ap.add_argument("--frames-per-launch", type=int, default=1)
    ap.add_argument("--variants", default=None,
                    help='JSON list of option dicts, e.g. [{"pop_on_miss": 1, "descent_cap": 8}] (replaces --occ)')
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401
    import visionaray_amd as va
    from visionaray_amd import scenes
    ctx = va.Context(0)
    prims = scenes.primitives(a.scene)
    prims["geom_id"] = np.arange(len(prims), dtype=np.uint32) % 3
    fn = va.face_normals(prims)
    dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), fn)
    dev.set_vertex_normals(np.repeat(fn, 3, axis=0))       # per-vertex binding with the face normals
    # the test suites' whitted spec: three plastic materials, three point lights
    m = np.zeros(3, va.PLASTIC_DTYPE)
    m[0] = ((0.2, 0.2, 0.2), 1.0, (0.8, 0.3, 0.2), 1.0, (1.0, 1.0, 1.0), 0.4, 32.0)
    m[1] = ((0.1, 0.1, 0.1), 0.5, (0.2, 0.7, 0.3), 0.9, (0.9, 0.9, 0.9), 0.2, 8.0)
    m[2] = ((0.05, 0.05, 0.1), 1.0, (0.3, 0.3, 0.9), 0.7, (1.0, 0.8, 0.6), 0.6, 64.5)
    lt = np.zeros(3, va.POINT_LIGHT_DTYPE)
    lt[0] = ((0.5, 2.0, 1.5), (1.0, 1.0, 1.0), 1.0, 1.0, 0.0, 0.0)
    lt[1] = ((-1.5, 1.0, 0.5), (1.0, 0.8, 0.6), 0.7, 1.0, 0.1, 0.05)
    lt[2] = ((0.2, 0.6, 0.3), (0.9, 0.9, 1.0), 0.8, 1.0, 0.2, 0.1)
    amb, bg = (0.4, 0.4, 0.4, 0.5), (0.1, 0.2, 0.3, 1.0)
    sh = va.shading(ctx, m, lt)
    cam, W, H = scenes.scene_camera(a.scene)
    rt = va.hip_buffer_rt(ctx, W, H)
    rt.alloc_multi_hit(16)
    kernels = {
        "simple_face": va.simple_kernel(dev, sh, bg=bg, ambient=amb),
        "simple_vertex": va.simple_kernel(dev, sh, binding=va.normals_per_vertex_binding, bg=bg, ambient=amb),
        "whitted_face_4": va.whitted_kernel(dev, sh, bg=bg, ambient=amb, num_bounces=4, epsilon=1e-3),
        "multi_hit_16": va.multi_hit_kernel(dev, sh, max_hits=16),
    }
    sched = va.hip_sched(ctx, async_frames=False)      # timed: frame() returns when the frame is done
    sp = va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt)
    F = a.frames_per_launch
    if F > 1:
        assert a.frames % F == 0, "--frames must be a multiple of --frames-per-launch"
        rtF = va.hip_buffer_rt(ctx, W, H * F)
        rtF.alloc_multi_hit(16)
        basis = cam.basis(W, H)

    def launch(k, n):
        if F == 1:
            sched.frame(k, sp, sync=False)
        else:
            va.render_batch(ctx, dev, rtF, [basis] * F, k, None, frame_num=n)
    variants = json.loads(a.variants) if a.variants else [{"waves_per_simd": int(x)} for x in a.occ.split(",")]
    for name, k in kernels.items():
        for v in variants:
            for opt, val in v.items():
                ctx.set_option(opt, val)
            occ = v.get("waves_per_simd", 0)
            try:
                for i in range(2):
                    launch(k, i)
                    ctx.sync()
                ctx.stats_reset()
                ctx.sync()
                t0 = time.perf_counter()
                for i in range(a.frames // F):
                    launch(k, i)
                ctx.sync()
                dt = time.perf_counter() - t0
                st = ctx.accum_stats()
                rays = int(st["rays"])
                print(json.dumps({"kernel": name, "occ": occ, "options": v, "scene": a.scene, "W": W, "H": H,
                                  "frames_per_launch": F,
                                  "ms_per_frame": round(dt / a.frames * 1e3, 3),
                                  "rays_per_frame": rays // a.frames,
                                  "Mrays_per_s": round(rays / dt / 1e6, 1)}), flush=True)
            except Exception as e:  # report and go on with the next variant
                print(json.dumps({"kernel": name, "occ": occ, "options": v, "error": str(e)}), flush=True)
            for opt in v:
                ctx.set_option(opt, 0)


if __name__ == "__main__":
    main()
