"""OBJ input measurement: parse throughput of vrh_obj_load on a generated
terrain, and (with --gpu) file -> first frame: load + GPU BVH build + one simple::kernel frame.

    python tools/obj_bench.py --grid 1000 [--gpu]      (prints one JSON line)
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--dir", default=None)
    a = ap.parse_args()
    import numpy as np
    import visionaray_amd as va
    from visionaray_amd import scenes
    d = a.dir or tempfile.mkdtemp(prefix="vrh_obj_")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "terrain.obj")
    t0 = time.perf_counter()
    obj, mtl = scenes.terrain_obj(a.grid)
    with open(path, "w") as f:
        f.write(obj)
    with open(os.path.join(d, "terrain.mtl"), "w") as f:
        f.write(mtl)
    gen_s = time.perf_counter() - t0
    size = os.path.getsize(path)
    best = 1e9
    for _ in range(a.reps):
        t0 = time.perf_counter()
        m = va.load_obj(path)
        best = min(best, time.perf_counter() - t0)
    res = {"what": "vrh_obj_load", "grid": a.grid, "bytes": size, "triangles": int(len(m.primitives)),
           "load_s": round(best, 4), "MB_per_s": round(size / best / 1e6, 1),
           "Mtri_per_s": round(len(m.primitives) / best / 1e6, 2), "gen_s": round(gen_s, 2)}
    if a.gpu:
        import torch  # noqa: F401  (HIP runtime before libvrh, as elsewhere)
        ctx = va.Context(0)
        W, H = 1920, 1080
        lights = np.zeros(1, va.POINT_LIGHT_DTYPE)
        lights[0] = ((0.5, 2.0, 1.5), (1.0, 1.0, 1.0), 1.0, 1.0, 0.0, 0.0)
        cam = va.camera()
        cam.perspective(45.0 * va.DEGREES_TO_RADIANS, W / H, 0.001, 1000.0)
        cam.look_at((0.3, 1.1, 1.6), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0))
        rt = va.hip_buffer_rt(ctx, W, H)
        sh = None
        times = []
        for _ in range(a.reps):
            ctx.sync()
            t0 = time.perf_counter()
            m = va.load_obj(path)
            t1 = time.perf_counter()
            dev = va.hip_index_bvh.gpu_build(ctx, m.primitives, m.geometric_normals)
            dev.set_vertex_normals(m.shading_normals)
            sh = va.shading(ctx, m.materials, lights)
            va.hip_sched(ctx).frame(va.simple_kernel(dev, sh, binding=va.normals_per_vertex_binding),
                                    va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt))
            ctx.sync()
            t2 = time.perf_counter()
            times.append((t2 - t0, t1 - t0, t2 - t1))
            dev.close()
            sh.close()
        best = min(times)
        res.update({"file_to_frame_s": round(best[0], 4), "load_part_s": round(best[1], 4),
                    "gpu_part_s": round(best[2], 4)})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
