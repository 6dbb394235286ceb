#!/usr/bin/env python3
"""bench.py -- Mrays/s (primary + 8-sample AO) of the MI355X traversal backend.

Workload (BASELINE.json configs[2], the config the metric is quoted on): the 1,002,528-triangle
procedural heightfield hf1M, binned-SAH index BVH, 1920x1080, one primary
closest-hit ray per pixel + 8 cosine-hemisphere any-hit AO rays (radius 0.1) per hit pixel.
A "step" is one frame.  Inputs (BVH, primitives, normals) are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Frames in flight (default F = 8): every persistent launch renders F frames (vrh_render_batch),
their tiles interleaved in the work queues, so no wave idles while the last tiles of a frame finish
-- the kernel-level tail is paid once per F frames.  Every frame is fully traced and written; the
last timed frames are checked against a separately rendered frame (frames_match_1gpu_frame).

N > 1: one process per GPU; the image is sharded by 8-row bands (band b -> rank b % N, SURVEY.md
§8e), each rank renders its packed shard of every frame, and the framebuffers are gathered to rank
0 over RCCL (torch.distributed "nccl"; prim ids + AO masks, 5 B/pixel, one gather per launch) and
un-interleaved there with the RGBA32F colour re-derived exactly (vrh_unshard).  Two launches are in
flight: launch k renders while launch k-1's gather runs on RCCL's stream; the last launch's gather
and un-interleave finish inside the timed region, so K steps = K complete frames on rank 0.  Total
work (K frames) is fixed as N grows, so scaling is strong.

Rank 0 prints one JSON line (contract in the task statement) with the roofline of the traversal
kernel (algorithmic bytes per SURVEY.md §8d from a counting pass, over the hipEvent kernel time of
the timed frames) and the CPU baseline (the reference's own SSE4 tiled_sched path, oracle/_ref,
timed on this host on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
TRI_BYTES, SPHERE_BYTES, INDEX_BYTES, NODE_BYTES = 64, 48, 4, 32
OUT_BYTES_PRIMARY = 24          # RGBA32F + u32 prim_id + f32 t per primary ray


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64, help="timed frames (default: two 32-frame launches)")
    ap.add_argument("--warmup", type=int, default=32, help="untimed frames (default: one launch)")
    ap.add_argument("--scene", default="hf1M", help="hf1M (C3, default) | hf10M (C4) | sph1M (C5)")
    ap.add_argument("--kernel", default=None, choices=["ao", "primary"], help="default: ao for triangles")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16, help="host cores for the CPU baseline")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL, the measured path) | gloo (host-staged; single-GPU rehearsal only)")
    ap.add_argument("--no-verify", action="store_true", help="skip the untimed check of the last frames against a 1-GPU frame")
    ap.add_argument("--frames-in-flight", type=int, default=32,
                    help="frames per persistent launch (vrh_render_batch, 1..32); every frame is still fully traced")
    return ap.parse_args()


def cpu_baseline(scene, kernel, threads):
    """Reference SSE4 tiled_sched<ray4> (oracle/_ref/vsnray_ref_bench) on a bounded sample:
    the same scene and camera at full resolution, 1 warm-up + 3 timed frames (~2-10 s)."""
    from oracle import oracle as O
    samples = 8 if kernel == "ao" else 0
    if os.path.exists(O.REF_BENCH_BIN):
        print(f"cpu baseline: reference tiled_sched, {threads} threads ...", file=sys.stderr, flush=True)
        try:
            r = O.ref_bench(scene, threads, 3, 1920, 1080, samples, timeout=150)
        except subprocess.TimeoutExpired:
            # tiled_sched's lost-wakeup race can stall a frame: one more try (CPU only)
            print("cpu baseline: timed out, retrying once", file=sys.stderr, flush=True)
            r = O.ref_bench(scene, threads, 3, 1920, 1080, samples, timeout=150)
        return {"value": round(r["mrays_per_s"], 3), "unit": "Mrays/s", "cores": threads, "kind": "reference",
                "sample": f"{scene} 1920x1080, {samples} AO spp, tiled_sched<basic_ray<simd::float4>> -O3 -msse4.1, "
                          f"median of 3 frames after 1 warm-up ({r['rays_per_frame']} rays/frame)"}
    # fallback: the plain-C restatement (scalar, OpenMP rows) on 1/8 of the image rows
    sc = O.make_scene(scene)
    cam = O.scene_camera(scene)
    mode = O.VO_MODE_AO if kernel == "ao" else O.VO_MODE_PRIMARY
    H = cam[5]
    rows = (0, H // 8)
    t0 = time.perf_counter()
    out = O.render(sc, cam, mode=mode, rows=rows, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(out["rays"] / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{scene} rows {rows[0]}-{rows[1]} of 1920x1080 ({out['rays']} rays), scalar C restatement"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}; using WORLD_SIZE", file=sys.stderr)

    # torch first: its HIP runtime is then the one libvrh.so binds to (one runtime per process)
    import torch
    import torch.distributed as dist

    import visionaray_amd as va
    from visionaray_amd import _capi, scenes

    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % max(ndev, 1))   # ranks > devices only in single-GPU rehearsals
    local = local % max(ndev, 1)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    kernel = args.kernel or ("ao" if not args.scene.startswith("sph") else "primary")

    # ---- CPU baseline (rank 0, N = 1 only), before any GPU work ------------------------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.scene, kernel, args.cpu_threads)
        except Exception as e:  # reported, never fatal for the GPU measurement
            cpu = {"value": None, "unit": "Mrays/s", "cores": args.cpu_threads, "kind": "reference",
                   "sample": f"failed: {e}"}

    # ---- scene: host build, upload (excluded from timing) --------------------------------------
    t0 = time.perf_counter()
    prims = scenes.primitives(args.scene)
    host = va.build_index_bvh(prims)
    build_s = time.perf_counter() - t0
    # one explicit stream shared by libvrh launches and torch/RCCL, so render -> gather -> unshard
    # are ordered on the device without host syncs
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = va.Context(local, stream=stream.cuda_stream)
    dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
    cam, W, H = scenes.scene_camera(args.scene)
    basis = cam.basis(W, H)
    kern = va.ao_kernel(dev) if kernel == "ao" else va.closest_hit_kernel(dev)
    kern_count = va.ao_kernel(dev, count_tests=True) if kernel == "ao" else va.closest_hit_kernel(dev, count_tests=True)

    # ---- frames in flight: every launch renders up to F frames (vrh_render_batch) -------------
    F = max(1, min(args.frames_in_flight, _capi.VRH_MAX_BATCH))

    def batches(k):
        return [F] * (k // F) + ([k % F] if k % F else [])

    # ---- framebuffers: full image on rank 0, packed shard per rank for N > 1 ------------------
    # Each rank writes its bands' prim ids and AO masks into ONE buffer per batch
    # [u32 prim ids of b frames | u8 masks of b frames] (5 B/pixel); one RCCL gather per batch moves
    # it to rank 0, which un-interleaves every frame and re-derives the RGBA32F colour exactly
    # (vrh_unshard) -- the full framebuffer (RGBA32F + prim ids) of every frame on rank 0.
    rows_max = _capi.VRH_BAND_ROWS * va.shard_bands(H, 0, world)
    n1 = rows_max * W                         # pixels of one frame's packed shard
    shard = _capi.vrh_shard(rank, world, 1, 0) if world > 1 else None
    nslots = 2                                # batch k renders while batch k - 1's gather runs
    bufs = {}                                 # batch size -> buffers

    def buffers(b):
        if b in bufs:
            return bufs[b]
        if world == 1:
            bufs[b] = {"rt": va.hip_buffer_rt(ctx, W, H * b)}
            return bufs[b]
        nb = n1 * b
        locs = [torch.empty((5 * nb,), dtype=torch.uint8, device="cuda") for _ in range(nslots)]
        d = {"locs": locs,
             "rts": [va.hip_buffer_rt(ctx, W, rows_max * b, wrap=(0, x.data_ptr(), 0, x.data_ptr() + 4 * nb))
                     for x in locs]}
        if rank == 0:
            d["gathered"] = [torch.empty((world, 5 * nb), dtype=torch.uint8, device="cuda") for _ in range(nslots)]
        bufs[b] = d
        return d

    fulls = []
    if world > 1 and rank == 0:
        fulls = [va.hip_buffer_rt(ctx, W, H, flags=_capi.VRH_RT_COLOR | _capi.VRH_RT_PRIM_ID | _capi.VRH_RT_OCC)
                 for _ in range(F)]

    def gather(b, slot):
        d = bufs[b]
        loc = d["locs"][slot]
        if args.dist_backend == "nccl":
            if rank == 0:
                return dist.gather(loc, gather_list=list(d["gathered"][slot].unbind(0)), dst=0, async_op=True)
            return dist.gather(loc, dst=0, async_op=True)
        # gloo rehearsal: stage through host memory, synchronously
        torch.cuda.synchronize()
        host = loc.cpu()
        if rank == 0:
            hg = torch.empty((world, host.numel()), dtype=torch.uint8)
            dist.gather(host, gather_list=list(hg.unbind(0)), dst=0)
            d["gathered"][slot].copy_(hg)
        else:
            dist.gather(host, dst=0)
        return None

    pending = []          # (work, batch size, slot) of gathers not yet waited for, oldest first

    def finish_one():
        work, b, slot = pending.pop(0)
        if work is not None:
            work.wait()   # the compute stream waits for the gather; the host does not block
        if rank == 0:
            g = bufs[b]["gathered"][slot].data_ptr()
            nb = n1 * b
            for f in range(b):
                va.unshard(ctx, W, H, world, fulls[f], prim_id_ptr=g + 4 * f * n1, occ_ptr=g + 4 * nb + f * n1,
                           shard_stride_bytes=5 * nb, kernel=kern)

    launch = [0]

    def run_batch(b):
        d = buffers(b)
        if world == 1:
            va.render_batch(ctx, dev, d["rt"], [basis] * b, kern, None)
            return
        slot = launch[0] % nslots
        launch[0] += 1
        # the slot's previous gather must be done before it is overwritten
        while any(pb == b and ps == slot for _, pb, ps in pending) or len(pending) >= nslots:
            finish_one()
        va.render_batch(ctx, dev, d["rts"][slot], [basis] * b, kern, shard)
        pending.append((gather(b, slot), b, slot))

    def drain():
        while pending:
            finish_one()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # ---- counting pass (untimed, one frame): box / primitive tests per ray ----------------------
    one_rows = rows_max if world > 1 else H
    rt_one = va.hip_buffer_rt(ctx, W, one_rows)
    va.render(ctx, dev, rt_one, basis, kern_count, shard)
    cstats = ctx.last_frame_stats()

    # ---- reference frame for the check below (rank 0, untimed): one vrh_render of the whole image
    # on another traversal schedule (the item loop; the step loop for sphere scenes, whose default
    # is the item loop) -- an independent code path, and a different kernel in the rocprof summary,
    # so every launch of the measured kernel is an F-frame launch
    ref = None
    if not args.no_verify and rank == 0:
        ctx.set_option("ao_schedule", 3 if args.scene.startswith("sph") else 4)
        ref_rt = va.hip_buffer_rt(ctx, W, H)
        va.render(ctx, dev, ref_rt, basis, kern, None)
        ref = ref_rt.download(t=False)
        ref_rt.close()
        ctx.set_option("ao_schedule", 0)

    for b in batches(args.warmup):
        run_batch(b)
    # every buffer the timed batches use (each batch size, each in-flight slot) is written once
    # before timing, whatever --warmup is
    for b in sorted(set(batches(args.steps))):
        for _ in range(nslots if world > 1 else 1):
            run_batch(b)
    drain()
    barrier()
    ctx.stats_reset()
    barrier()
    t0 = time.perf_counter()
    for b in batches(args.steps):
        run_batch(b)
    drain()               # the last batch's gather and un-interleave are inside the timed region
    barrier()
    elapsed = time.perf_counter() - t0
    acc = ctx.accum_stats()
    last_b = batches(args.steps)[-1]

    # ---- the timed frames are right: N > 1 gathered frames (rank 0) equal a 1-GPU frame ---------
    verified = None
    if ref is not None:
        b = ref
        if world > 1:
            outs = [fulls[f].download(t=False) for f in range(last_b)]
        else:
            a = bufs[last_b]["rt"].download(t=False)
            outs = [{k: v[f * W * H:(f + 1) * W * H] for k, v in a.items()} for f in range(last_b)]
        verified = bool(all((o[k].view("u1") == b[k].view("u1")).all() for o in outs for k in ("color", "prim_id", "occ")))
    barrier()

    # ---- aggregate over ranks -------------------------------------------------------------------
    local_vals = torch.tensor([elapsed, float(acc["rays"]), acc["kernel_ms_total"], float(acc["timed_frames"]),
                               float(cstats["box_tests"]), float(cstats["prim_tests"]), float(cstats["rays"]),
                               float(cstats["hits"])], dtype=torch.float64, device="cuda")
    if world > 1:
        mx = local_vals.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = local_vals.clone()
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    else:
        mx = sm = local_vals
    t_max = float(mx[0])
    total_rays = float(sm[1])
    mrays = total_rays / t_max / 1e6

    if rank == 0:
        # algorithmic bytes: 32 B per box test (a 64-B child pair per inner visit),
        # (S_prim + 4 index) B per primitive test, 24 B of output per primary ray
        s_prim = TRI_BYTES if args.scene.startswith("hf") or args.scene == "cornell12" else SPHERE_BYTES
        n_box, n_prim, n_rays = float(sm[4]), float(sm[5]), float(sm[6])
        primary_rays = W * H
        bytes_frame = NODE_BYTES * n_box + (s_prim + INDEX_BYTES) * n_prim + OUT_BYTES_PRIMARY * primary_rays
        bytes_per_ray = bytes_frame / n_rays
        # dominant kernel = the traversal kernel; per-launch (F frames) algorithmic bytes over its mean
        # hipEvent time
        k_ms_mean = float(local_vals[2]) / max(float(local_vals[3]), 1.0)    # rank 0's launches
        local_bytes = bytes_per_ray * float(acc["rays"]) / max(float(acc["timed_frames"]), 1.0)
        achieved = local_bytes / (k_ms_mean * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                with open(pmc) as f:
                    pm = json.load(f)
                if (pm.get("scene") == args.scene and pm.get("kernel") == kernel and pm.get("gpus") == 1 and world == 1
                        and pm.get("frames_per_launch", 1) == F):
                    traffic = pm.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        # what actually limits the kernel (PMC, tools/profile_mem.sh): busy fractions of the
        # vector-memory address (TA) and data (TD) units, when measured for this configuration
        limiter = None
        pmm = os.path.join(ROOT, "profiles", "pmc_mem.json")
        if os.path.exists(pmm) and world == 1:
            try:
                with open(pmm) as f:
                    pm = json.load(f)
                if pm.get("scene") == args.scene and pm.get("kernel") == kernel and pm.get("frames_per_launch") == F:
                    limiter = {"unit": "vector-memory pipeline (L1 / TA address / TD data)",
                               "td_busy": round(pm["td_busy_frac"], 3), "ta_busy": round(pm["ta_busy_frac"], 3),
                               "l1_hit": round(1.0 - pm["l1_to_l2_reads_per_access"], 3),
                               "td_stalled_on_l1": (round(pm["td_stalled_on_l1_frac"], 3)
                                                    if pm.get("td_stalled_on_l1_frac") is not None else None),
                               "source": "profiles/pmc_mem.json (rocprofv3 --pmc, same workload)"}
            except Exception:
                limiter = None
        line = {
            "metric": "Mrays/s (primary + 8-sample AO)" if kernel == "ao" else "Mrays/s (primary)",
            "value": round(mrays, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (SURVEY.md Appendix A procedural scene, deterministic)",
            "config": {
                "workload": f"{args.scene} {W}x{H} 1 spp primary" + (" + 8 AO any-hit rays/hit (r=0.1)" if kernel == "ao" else ""),
                "scene": args.scene, "primitives": int(len(prims)), "bvh_nodes": int(len(host.nodes)),
                "width": W, "height": H, "ao_samples": 8 if kernel == "ao" else 0,
                "rays_per_frame": int(n_rays), "parallelism": f"image-tile shard x{world}" + (" + RCCL gather" if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": "render_unified_kernel (traversal)", "kernel_ms_mean": round(k_ms_mean, 4),
                "frames_per_launch": F, "kernel_ms_per_frame": round(float(local_vals[2]) / args.steps, 4),
                "bytes_per_ray": round(bytes_per_ray, 1), "box_tests_per_ray": round(n_box / n_rays, 3),
                "prim_tests_per_ray": round(n_prim / n_rays, 3),
                "measured_limiter": limiter,
            },
            "cpu_baseline": cpu,
            "host_build_s": round(build_s, 3),
            "frames_in_flight": F,
            "frames_match_1gpu_frame": verified,
        }
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
