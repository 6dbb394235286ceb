"""Time-to-first-frame: host binned-SAH build + upload vs GPU linear-BVH build (vrh_scene_build),
and the traversal rate on both trees (SURVEY.md §8f rank 2 measurement).

    python tools/build_bench.py [scene ...]      -> one JSON line per scene (also gpurun_out/build_bench.jsonl)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import visionaray_amd as va  # noqa: E402
from visionaray_amd import scenes  # noqa: E402

os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
ctx = va.Context(0)


def rate(dev, name, frames=10):
    cam, W, H = scenes.scene_camera(name)
    prims_tri = not name.startswith("sph")
    k = va.ao_kernel(dev) if prims_tri else va.closest_hit_kernel(dev)
    rt = va.hip_buffer_rt(ctx, W, H)
    basis = cam.basis(W, H)
    va.render(ctx, dev, rt, basis, k)
    ctx.stats_reset()
    for _ in range(frames):
        va.render(ctx, dev, rt, basis, k)
    a = ctx.accum_stats()
    return a["rays"] / a["kernel_ms_total"] / 1e3, a["kernel_ms_total"] / a["timed_frames"]


for name in sys.argv[1:] or ["hf1M", "sph1M", "hf10M"]:
    prims = scenes.primitives(name)
    nrm = scenes.normals_for(prims)
    t0 = time.perf_counter()
    host = va.build_index_bvh(prims)
    t1 = time.perf_counter()
    dev_sah = va.hip_index_bvh(ctx, host, nrm)
    ctx.sync() if hasattr(ctx, "sync") else None
    t2 = time.perf_counter()
    sah_rate, sah_ms = rate(dev_sah, name)
    sah_cost = va.sah_cost(host.nodes)
    dev_sah.close()
    va.hip_index_bvh.gpu_build(ctx, prims, nrm).close()          # warm-up (code objects, allocator)
    t3 = time.perf_counter()
    dev_gpu = va.hip_index_bvh.gpu_build(ctx, prims, nrm)
    t4 = time.perf_counter()
    gpu_rate, gpu_ms = rate(dev_gpu, name)
    nodes, _ = dev_gpu.download_bvh()
    rec = {"scene": name, "prims": len(prims),
           "host_sah_build_s": round(t1 - t0, 4), "host_upload_s": round(t2 - t1, 4),
           "gpu_build_wall_s": round(t4 - t3, 4), "gpu_build_kernels_ms": round(dev_gpu.info["build_ms"], 3),
           "speedup_time_to_scene": round((t2 - t0) / (t4 - t3), 1),
           "sah_cost_host": round(sah_cost, 4), "sah_cost_gpu": round(va.sah_cost(nodes), 4),
           "mrays_s_sah_tree": round(sah_rate, 1), "mrays_s_gpu_tree": round(gpu_rate, 1),
           "frame_ms_sah_tree": round(sah_ms, 4), "frame_ms_gpu_tree": round(gpu_ms, 4),
           "depth_sah": host.max_depth, "depth_gpu": dev_gpu.info["max_depth"]}
    line = json.dumps(rec)
    print(line, flush=True)
    with open(os.path.join(ROOT, "gpurun_out", "build_bench.jsonl"), "a") as f:
        f.write(line + "\n")
