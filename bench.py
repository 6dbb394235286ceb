#!/usr/bin/env python3
"""bench.py -- Mrays/s (primary + 8-sample AO) of the MI355X traversal backend.

Workload (BASELINE.json configs[2], the config the metric is quoted on): the 1,002,528-triangle
procedural heightfield hf1M, binned-SAH index BVH, 1920x1080, one primary
closest-hit ray per pixel + 8 cosine-hemisphere any-hit AO rays (radius 0.1) per hit pixel.
A "step" is one frame.  Inputs (BVH, primitives, normals) are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

--gpus N > 1 without a launcher (no WORLD_SIZE): bench.py starts the N ranks itself as child processes
before anything touches the GPU (launch_plan / spawn_ranks); with fewer GPUs than N, or WORLD_SIZE
disagreeing with --gpus, it exits 2 with a message and prints no line.

Frames: every frame has its own frame number (vrh_render's frame_num -> its own AO sample set,
as the reference reseeds per frame, cuda_sched.inl:38-45, 79): the W warm-up frames are numbers
1..W, the K timed frames W+1..W+K; frame 0 and frame 3 are rendered once, untimed, and checked
against the reference's fixtures (tests/golden).

Frames in flight: the K timed frames run as K / F persistent launches of F frames each
(vrh_render_batch; F = the largest divisor of K not above --frames-in-flight), so the kernel's
tail is paid once per launch.  `value` is K frames' rays over the wall time of the timed region.
The hip_sched::frame path -- one synchronous launch per frame, as the reference's scheduler
issues frames -- is measured separately over --single-frames frames (median): single_frame_*.
single_frame_async_* is the same frame() path with asynchronous issue (VRH_OPT_ASYNC_FRAMES, the
cuda_sched model): --single-frames back-to-back calls, one final sync, rate over the hipEvent span.
The timed frames share the scene camera (their AO samples differ); moving_camera_* repeats the
timed launches with the eye orbiting --moving-camera degrees per frame (default 0.5: no two frames
share primary rays), reported beside the headline.

N > 1: one process per GPU, one libvrh render group over RCCL (vrh_group_join, the id broadcast
by torch.distributed): each rank renders its image-tile shard (8-row bands, band b -> rank b % N,
SURVEY.md §8e) of every frame and libvrh gathers the packed shards to rank 0 with ncclSend /
ncclRecv on its own stream and un-interleaves them there (vrh_render_sharded).  K frames are
fixed as N grows: scaling "strong".

Rank 0 prints one JSON line (the contract of the task statement) with:
  * roofline: the unit that binds the traversal kernel is the vector-memory path (L1 / TA / TD:
    TD busy 94-97 % of the launch, PMC in profiles/r02_*), so `achieved` is the kernel's vector-L1
    request rate -- rocprofv3's TCP_TOTAL_CACHE_ACCESSES of the committed PMC pass of this exact
    command (profiles/pmc_traffic_F<F>.json) x 16 B per launch over the live hipEvent launch time -- and
    `peak` the highest request rate of the kernel's access shape (per-lane dependent 64-B record
    gathers) on the microbenchmark tools/micro/l1_roof.hip (profiles/l1_roof.json).  The SURVEY
    §8d algorithmic HBM bytes are kept as roofline.hbm_algorithmic (informational);
  * cpu_baseline: the reference's own SSE4 tiled_sched path (oracle/_ref, built from
    /root/reference by oracle/Makefile) on a bounded sample at threads = the CPUs the process may use
    (cgroup quota) at most: the best of a cores/4, cores/2, cores - 1, cores sweep, 3 runs per point of 7 frames each,
    the host's core count, quota and model, and the retries / stall seconds of tiled_sched stalls.

Settle: after the W warm-up steps, untimed launches of the timed shape run for --settle-ms (300 ms) of
wall time so that the timed launches run at the GPU's sustained clocks (the line's `settle` object).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
TRI_BYTES, SPHERE_BYTES, INDEX_BYTES, NODE_BYTES = 64, 48, 4, 32
OUT_BYTES_PRIMARY = 24          # RGBA32F + u32 prim_id + f32 t per primary ray
GROUP_TIMEOUT_MS = 60000        # N > 1: deadline of every wait on a peer rank (join, exchange, sync)
L1_REQ_BYTES = 16               # one vector-L1 request (TCP access) = one lane's 16-B piece (tools/l1_roof.py)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64, help="timed frames")
    ap.add_argument("--warmup", type=int, default=32, help="untimed frames before the timed region")
    ap.add_argument("--scene", default="hf1M", help="hf1M (C3, default) | hf10M (C4) | sph1M (C5)")
    ap.add_argument("--kernel", default=None, choices=["ao", "primary"], help="default: ao for triangles")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="host threads for the CPU baseline (default: the best of a cores/4, cores/2, cores - 1, "
                         "cores sweep, cores = the CPUs the process may use)")
    ap.add_argument("--no-verify", action="store_true", help="skip the untimed checks against the fixtures")
    ap.add_argument("--no-user-kernel", action="store_true",
                    help="skip the user-kernel leg (hf1M AO at N=1: hip_kernels.h device lambda, 32 frames per launch)")
    ap.add_argument("--frames-in-flight", type=int, default=32,
                    help="max frames per persistent launch (vrh_render_batch, 1..32)")
    ap.add_argument("--single-frames", type=int, default=10, help="frames of the hip_sched::frame leg (median)")
    ap.add_argument("--moving-camera", type=float, default=0.5,
                    help="degrees of camera orbit per frame in an extra moving-camera leg after the timed region "
                         "(0: no such leg); its launches have the timed launches' shape")
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed launches of the timed shape for this long after the warm-up steps "
                         "(GPU clock ramp), 0 = none")
    ap.add_argument("--gather-ids", action="store_true",
                    help="N > 1 / --shards: gather prim ids + AO masks with the colour (5 B per pixel on the wire, not 1)")
    ap.add_argument("--shards", type=int, default=0,
                    help="image-tile shards of the render group (0 = one per rank); > ranks: a rank renders several")
    return ap.parse_args()


def host_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return {"cpu_model": model, "host_cpus": os.cpu_count(), "cpus_available": avail}


def cgroup_cpu_quota():
    """CPUs the cgroup lets this process use (cpu.max quota / period), or None without a quota."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def usable_cpus(info):
    """CPUs this process can actually run on: the cgroup quota (rounded down, at least 1) when there is
    one, else the affinity mask.  The baseline's worker-thread count is reported separately."""
    q = info.get("cgroup_cpu_quota")
    avail = info.get("cpus_available") or 1
    return max(1, min(avail, int(q))) if q else avail


CPU_ATTEMPT_TIMEOUT_S = 90
CPU_FRAMES = 7                  # timed frames per sweep point (median), after 1 warm-up frame


CPU_RUNS = 3                    # runs per sweep point; the fastest one counts (a run can only be slowed)


def cpu_sweep_points(cores, threads=None):
    """Worker-thread counts of the CPU baseline: --cpu-threads alone, else cores/4, cores/2, cores - 1
    and cores -- never above the CPUs the process may use (oversubscribed points measured up to 3x
    apart between sessions)."""
    if threads:
        return [threads]
    return sorted({max(1, cores // 4), max(1, cores // 2), max(1, cores - 1), cores})


def cpu_baseline(scene, kernel, threads=None):
    """Reference SSE4 tiled_sched<ray4> (oracle/_ref/vsnray_ref_bench) on a bounded sample: the same
    scene and camera at full resolution, 1 warm-up + CPU_FRAMES timed frames per run, the median
    frame; CPU_RUNS runs per point, the fastest counts.  Points: cores/4, cores/2, cores - 1 and cores
    (the CPUs this process may use: the cgroup quota, else the affinity mask), never more.  `value` is
    the best point.  At threads = cores the workers alone fill the quota, so any other thread of the
    container (the Python parent, the HIP runtime) makes CFS throttle all of them: round 6 measured
    93.4 and 75.1 Mrays/s there in two sessions while 8 threads gave 43.21 / 43.13 (profiles/r06/cpu/),
    hence cores - 1 beside it and the best of the sweep as `value`.  Each point's min / max frame rate
    is reported.  tiled_sched can lose a worker's wake-up (tiled_sched.inl:181 waits
    without a predicate against the notify_all at :386) and stall a frame for good: a run that passes
    CPU_ATTEMPT_TIMEOUT_S is killed and tried once more, and the line records the retries and the
    seconds lost to stalls."""
    from oracle import oracle as O
    samples = 8 if kernel == "ao" else 0
    info = host_info()
    info["cgroup_cpu_quota"] = cgroup_cpu_quota()
    cores = usable_cpus(info)
    info["cores_note"] = ("cores = the CPUs the process may use (cgroup quota, else affinity); value = the best "
                          "sweep point, threads = its worker threads (never above cores)")
    if os.path.exists(O.REF_BENCH_BIN):
        counts = cpu_sweep_points(cores, threads)
        sweep, retries, stall_s = [], 0, 0.0
        for n in counts:
            print(f"cpu baseline: reference tiled_sched, {n} threads ...", file=sys.stderr, flush=True)
            point = {"threads": n, "value": None, "runs": [], "retries": 0, "stall_s": 0.0}
            for run in range(CPU_RUNS):
                for attempt in range(2):
                    t0 = time.perf_counter()
                    try:
                        r = O.ref_bench(scene, n, CPU_FRAMES, 1920, 1080, samples, timeout=CPU_ATTEMPT_TIMEOUT_S)
                    except subprocess.TimeoutExpired:
                        lost = time.perf_counter() - t0
                        print(f"cpu baseline: {n} threads stalled ({lost:.0f} s, tiled_sched lost wake-up)",
                              file=sys.stderr, flush=True)
                        point["stall_s"] = round(point["stall_s"] + lost, 1)
                        if attempt == 0:
                            point["retries"] += 1
                        continue
                    rpf = r["rays_per_frame"]
                    point["runs"].append(round(r["mrays_per_s"], 3))
                    if point["value"] is None or r["mrays_per_s"] > point["value"]:
                        point["value"] = round(r["mrays_per_s"], 3)
                        point["rays_per_frame"] = rpf
                        if r.get("min_s"):
                            # frame-rate spread of the run: slowest and fastest of its timed frames
                            point["min"] = round(rpf / r["max_s"] / 1e6, 3)
                            point["max"] = round(rpf / r["min_s"] / 1e6, 3)
                            point["spread"] = round((r["max_s"] - r["min_s"]) / r["median_s"], 4)
                    break
            retries += point["retries"]
            stall_s += point["stall_s"]
            sweep.append(point)
        done = [p for p in sweep if p["value"] is not None]
        if not done:
            raise RuntimeError(f"every reference run stalled: {sweep}")
        at = max(done, key=lambda p: p["value"])
        at_cores = next((p["value"] for p in done if p["threads"] == cores), None)
        return {"value": at["value"], "unit": "Mrays/s", "cores": cores, "threads": at["threads"],
                "kind": "reference",
                "sample": f"{scene} 1920x1080, {samples} AO spp, tiled_sched<basic_ray<simd::float4>> -O3 -msse4.1, "
                          f"best of a worker-thread sweep {counts} within the {cores} CPUs the process may use "
                          f"(the fastest of {CPU_RUNS} runs per point, each the median of {CPU_FRAMES} frames after 1 "
                          f"warm-up; {at['rays_per_frame']} rays/frame)",
                "sweep": sweep, "value_at_threads_eq_cores": at_cores,
                "retries": retries, "stall_s": round(stall_s, 1), **info}
    # fallback: the plain-C restatement (scalar, OpenMP rows) on 1/8 of the image rows
    threads = threads or min(16, info["cpus_available"] or 1)
    sc = O.make_scene(scene)
    cam = O.scene_camera(scene)
    mode = O.VO_MODE_AO if kernel == "ao" else O.VO_MODE_PRIMARY
    H = cam[5]
    rows = (0, H // 8)
    t0 = time.perf_counter()
    out = O.render(sc, cam, mode=mode, rows=rows, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": round(out["rays"] / dt / 1e6, 3), "unit": "Mrays/s", "cores": min(threads, usable_cpus(info)),
            "threads": threads, "kind": "port",
            "sample": f"{scene} rows {rows[0]}-{rows[1]} of 1920x1080 ({out['rays']} rays), scalar C restatement",
            "retries": 0, "stall_s": 0.0, **info}


def user_program_run(prog, W, H, n_rays):
    """median frame time of tests/cpp/user_kernels.hip's `bench` mode built as build/tests/<prog>; null
    when the program is absent"""
    exe = os.path.join(ROOT, "build", "tests", prog)
    if not os.access(exe, os.X_OK):
        return None
    try:
        r = subprocess.run([exe, "bench", "708", str(W), str(H), "/tmp", "4", "32"], capture_output=True,
                           text=True, timeout=180)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    rec = None
    for ln in r.stdout.splitlines():
        if ln.startswith("{") and "frame_ms_median" in ln:
            rec = json.loads(ln)
    if r.returncode != 0 or rec is None:
        return {"error": f"rc {r.returncode}"}
    ms = float(rec["frame_ms_median"])
    # the lambda traces the built-in kernel's rays: the same primary rays, 8 AO rays per hit
    return {"mrays": round(n_rays / (ms * 1e-3) / 1e6, 1), "frame_ms_median": ms,
            "frames_per_launch": rec["frames_per_launch"], "launches": rec["launches"],
            # the instance the launch took (register target: 0 = the compiler's own), its one-wave blocks
            # per CU and the LDS stack entries per thread (hip_kernels.h launch_user_render)
            "launch": rec.get("launch"),
            "program": "build/tests/%s bench 708 %d %d /tmp 4 32" % (prog, W, H)}


def user_kernel_leg(W, H, n_rays):
    """The same workload through a user kernel: the AO lambda of tests/cpp/user_kernels.hip (ao/main.cpp's
    kernel with random_sampler directions, include/visionaray_hip/hip_kernels.h, compiled by hipcc) on
    hip_sched::frames, 32 frames per launch, median over 4 launches -- the path a Visionaray program with
    its own kernel takes.  Run after the timed region, in a child process; null when the program is absent."""
    leg = user_program_run("user_kernels", W, H, n_rays)
    if leg is None or "error" in leg:
        return leg
    leg["kernel"] = "AO device lambda (ao/main.cpp's, random_sampler) via hip_kernels.h on hip_sched::frames"
    # the same program built with deferred any_hit calls (hip_kernels.h VRH_USER_DEFER=1: each tile's
    # kernel runs record / trace / replay, the any_hit rays traced as one pool): the same frames
    leg["deferred"] = user_program_run("uk_defer", W, H, n_rays)
    rec = {"frames_per_launch": leg["frames_per_launch"]}
    ms = leg["frame_ms_median"]
    # roofline of the user kernel, as the built-in's: the vector-L1 requests of the committed PMC pass of
    # this program (profiles/pmc_user_lambda.json; the hash of libvrh's and the user-kernel headers'
    # sources checked) x 16 B over the live launch time (median wall time of a 32-frame frames() launch:
    # the kernel plus its launch, an upper bound)
    pmc = load_json(os.path.join(ROOT, "profiles", "pmc_user_lambda.json")) or {}
    roof = load_json(os.path.join(ROOT, "profiles", "l1_roof.json"))
    from visionaray_amd.buildinfo import user_kernel_source_sha256
    if (pmc.get("l1_requests_per_launch") and pmc.get("frames_per_launch") == rec["frames_per_launch"]
            and pmc.get("user_kernel_source_sha256") == user_kernel_source_sha256() and roof):
        launch_s = ms * 1e-3 * rec["frames_per_launch"]
        achieved = pmc["l1_requests_per_launch"] * L1_REQ_BYTES / launch_s / 1e9
        sq = load_json(os.path.join(ROOT, "profiles", "pmc_sq_lambda.json")) or {}
        if sq.get("user_kernel_source_sha256") != user_kernel_source_sha256():
            sq = {}
        leg["roofline"] = {"bound": "vmem-l1", "unit": "GB/s", "achieved": round(achieved, 1), "peak": roof.get("peak_gbs"),
                           "frac": round(achieved / roof["peak_gbs"], 4), "td_busy_frac": round(pmc["td_busy_frac"], 4),
                           "l1_requests_per_launch": pmc["l1_requests_per_launch"],
                           "waves_per_launch": pmc.get("waves_per_launch"),
                           "lane_utilisation_valu": sq.get("lane_utilisation_valu"),
                           "valu_insts_per_ray": sq.get("valu_insts_per_ray"),
                           "source": "profiles/pmc_user_lambda.json, profiles/pmc_sq_lambda.json, profiles/l1_roof.json"}
    else:
        leg["roofline"] = None
    return leg


def frames_per_launch(steps, cap):
    """The largest divisor of `steps` that is <= cap (every timed launch has the same size)."""
    cap = max(1, min(cap, 32))
    return max(d for d in range(1, cap + 1) if steps % d == 0)


def load_json(path):
    try:
        with open(path) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


LAUNCH_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def launch_plan(gpus, env, device_count):
    """What this process does for --gpus `gpus` under environment `env` on a node with `device_count`
    GPUs (counted without initialising the GPU): ("run", None) -- this process is one rank (N = 1, or a
    rank started by torch.distributed.run / by this launcher); ("spawn", [env of rank 0..N-1]) -- no
    launcher ran: start the N ranks as child processes (nothing here has touched the GPU); or ("error",
    message) -- a run that would measure something other than N GPUs (more ranks than GPUs, WORLD_SIZE
    and --gpus disagreeing), which must never print a line."""
    if gpus < 1:
        return "error", f"--gpus {gpus}: at least one GPU"
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            return "error", (f"WORLD_SIZE={world} but --gpus {gpus}: the line would report {world} GPUs for a "
                             f"{gpus}-GPU run; launch with --nproc-per-node {gpus}")
        local = int(env.get("LOCAL_RANK", env.get("RANK", "0")))
        if world > 1 and local >= device_count:
            return "error", (f"rank with LOCAL_RANK={local} of {world} ranks, but this node has {device_count} "
                             f"GPU(s): one process per GPU is required (ranks may not share a GPU)")
        return "run", None
    if gpus == 1:
        return "run", None
    if device_count < gpus:
        return "error", (f"--gpus {gpus}, but this node has {device_count} GPU(s): refusing to measure fewer "
                         f"GPUs than asked (one process per GPU)")
    port = int(env.get("MASTER_PORT", "0")) or free_port()
    envs = []
    for r in range(gpus):
        e = dict(env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(gpus), "LOCAL_WORLD_SIZE": str(gpus),
                  "MASTER_ADDR": env.get("MASTER_ADDR", "127.0.0.1"), "MASTER_PORT": str(port)})
        envs.append(e)
    return "spawn", envs


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(envs, argv, grace_s=None):
    """Start one child process per rank (this process never touches the GPU and does not exec), rank 0's
    stdout (the JSON line) passed through; the others' stdout goes to stderr.  When a rank fails, the
    rest end through their group deadlines (GROUP_TIMEOUT_MS); whatever still runs `grace_s` later is
    killed by its own process group.  Returns the first non-zero exit status (0 when every rank passed)."""
    import signal
    grace_s = grace_s if grace_s is not None else 3 * GROUP_TIMEOUT_MS / 1e3 + 30
    procs = []
    for r, e in enumerate(envs):
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=e,
                                      stdout=None if r == 0 else sys.stderr.fileno(), start_new_session=True))
    first_bad, t_fail = 0, None
    while True:
        live = [p for p in procs if p.poll() is None]
        for p in procs:
            if p.returncode not in (None, 0) and not first_bad:
                first_bad, t_fail = p.returncode, time.monotonic()
                print(f"bench launcher: rank {procs.index(p)} exited with {p.returncode}; waiting up to "
                      f"{grace_s:.0f} s for the other ranks", file=sys.stderr, flush=True)
        if not live:
            break
        if t_fail is not None and time.monotonic() - t_fail > grace_s:
            for p in live:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
            for p in live:
                p.wait()
            break
        time.sleep(0.05)
    return first_bad if first_bad else (1 if any(p.returncode for p in procs) else 0)


def device_count():
    """GPUs of this node without initialising the GPU (torch.cuda.device_count does not, on this image)."""
    import torch
    return torch.cuda.device_count()


def main():
    args = parse()
    action, info = launch_plan(args.gpus, os.environ, device_count() if args.gpus > 1 or
                               int(os.environ.get("WORLD_SIZE", "1")) > 1 else 1)
    if action == "error":
        print(f"bench.py: error: {info}", file=sys.stderr, flush=True)
        sys.exit(2)
    if action == "spawn":
        print(f"bench launcher: starting {len(info)} ranks (no WORLD_SIZE in the environment)", file=sys.stderr,
              flush=True)
        sys.exit(spawn_ranks(info, sys.argv[1:]))
    # the JSON line is the only thing on stdout: native libraries (RCCL prints a version banner at
    # communicator init) write to fd 1 directly, so fd 1 becomes stderr and the line goes to a dup
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # torch first: its HIP runtime (and RCCL) is then the one libvrh.so binds to (one per process)
    import numpy as np
    import torch
    import torch.distributed as dist

    import visionaray_amd as va
    from visionaray_amd import _capi, scenes

    torch.cuda.set_device(local)
    if world > 1:
        import datetime
        dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(milliseconds=3 * GROUP_TIMEOUT_MS))

    kernel = args.kernel or ("ao" if not args.scene.startswith("sph") else "primary")

    # ---- CPU baseline (rank 0, N = 1 only), before any GPU work ------------------------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.scene, kernel, args.cpu_threads)
        except Exception as e:  # reported, never fatal for the GPU measurement
            cpu = {"value": None, "unit": "Mrays/s", "cores": args.cpu_threads or 0, "kind": "reference",
                   "sample": f"failed: {e}", **host_info()}

    # ---- scene: host build, upload (excluded from timing) --------------------------------------
    t0 = time.perf_counter()
    prims = scenes.primitives(args.scene)
    host = va.build_index_bvh(prims)
    build_s = time.perf_counter() - t0
    ctx = va.Context(local)
    dev = va.hip_index_bvh(ctx, host, scenes.normals_for(prims))
    cam, W, H = scenes.scene_camera(args.scene)
    basis = cam.basis(W, H)
    mk = va.ao_kernel if kernel == "ao" else va.closest_hit_kernel
    kern, kern_count = mk(dev), mk(dev, count_tests=True)
    rays_key = "rays"

    F = frames_per_launch(args.steps, args.frames_in_flight)
    launches = args.steps // F

    # ---- render paths -----------------------------------------------------------------------
    group = None
    grouped = world > 1 or args.shards > 1     # one GPU with --shards S: a one-rank group (rehearsal)
    if world > 1:
        # the group id travels over torch.distributed once; the data path is libvrh + RCCL
        uid = torch.zeros(va.GROUP_ID_BYTES, dtype=torch.uint8, device="cuda")
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(va.render_group.unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        # every wait on a peer has a deadline (vrh_group_join_timeout): a dead rank ends the others with an
        # error instead of a hang
        group = va.render_group(ctx, world, rank, bytes(uid.cpu().numpy().tobytes()), timeout_ms=GROUP_TIMEOUT_MS)
    elif grouped:
        group = va.render_group(ctx, 1, 0, va.render_group.unique_id())
    full_rts = {}

    # N > 1: the root assembles the frame's colour (the AO example's product); its built-in colour
    # crosses the wire as one byte per pixel (hit + occluded-sample count).  --gather-ids adds the
    # prim ids and AO masks (5 B per pixel).
    gather_fields = _capi.VRH_RT_COLOR | ((_capi.VRH_RT_PRIM_ID | _capi.VRH_RT_OCC) if args.gather_ids else 0)

    def target(b):
        """Full-image target of b frames (rank 0; every rank for N = 1)."""
        if b not in full_rts:
            flags = _capi.VRH_RT_ALL if not grouped else gather_fields
            full_rts[b] = va.hip_buffer_rt(ctx, W, H * b, flags=flags) if (world == 1 or rank == 0) else None
        return full_rts[b]

    next_frame = [1]

    def run_batch(b):
        fn = next_frame[0]
        next_frame[0] += b
        if not grouped:
            va.render_batch(ctx, dev, target(b), [basis] * b, kern, None, frame_num=fn)
        else:
            group.render(dev, kern, target(b), [basis] * b, frame_num=fn, shards=args.shards, fields=gather_fields)
        return fn

    def sync():
        if group is not None:
            group.sync()
        ctx.sync()

    def barrier():
        sync()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # ---- counting pass (untimed, one frame on rank 0's whole image): tests and L1 lines per ray --
    rt_one = va.hip_buffer_rt(ctx, W, H)
    va.render(ctx, dev, rt_one, basis, kern_count, None, frame_num=0)
    cstats = ctx.last_frame_stats()

    # ---- fixtures: frame 0 and frame 3 against the reference's outputs (untimed) ---------------
    verify = {}
    if not args.no_verify and rank == 0:
        golden = load_json(os.path.join(ROOT, "tests", "golden", "golden.json")) or {}
        for case, fnum in ((args.scene, 0), (f"frame3_{args.scene}", 3)):
            g = golden.get(case)
            path = os.path.join(ROOT, "tests", "golden", case + ".npz")
            if not g or not os.path.exists(path) or (kernel == "ao") != (g.get("ao_rays", 0) > 0):
                continue
            va.render(ctx, dev, rt_one, basis, kern, None, frame_num=fnum)
            out = rt_one.download()
            ref = np.load(path)
            pix = ref["pixels"]
            ok = all(np.array_equal(out[k][pix].view(np.uint8), ref[k].view(np.uint8))
                     for k in ("prim_id", "t", "occ", "color") if k in ref)
            verify[f"frame{fnum}_matches_reference_sample"] = bool(ok)
    rt_one.close()

    # ---- warm-up, then every timed batch size is run once so first-touch costs stay out ----------
    for _ in range(args.warmup // F):
        run_batch(F)
    for _ in range(args.warmup % F):
        run_batch(1)
    run_batch(F)
    # settle: the GPU ramps its clocks over the first ~0.1-0.3 s of sustained work, and W warm-up steps
    # of 0.2-1.1 ms frames are far shorter than that; untimed launches of the timed shape until
    # --settle-ms of wall time have passed (reported in the line), so the timed launches run at the
    # clocks every later launch runs at
    settle_t0 = time.perf_counter()
    settle_launches = 0
    while (time.perf_counter() - settle_t0) * 1e3 < args.settle_ms:
        run_batch(F)
        settle_launches += 1
        if settle_launches % 8 == 0:
            sync()
    barrier()
    settle = {"ms": round((time.perf_counter() - settle_t0) * 1e3, 1), "launches": settle_launches,
              "frames_per_launch": F}
    ctx.stats_reset()
    barrier()
    first_timed = next_frame[0]
    t0 = time.perf_counter()
    for _ in range(launches):
        run_batch(F)
    barrier()
    elapsed = time.perf_counter() - t0
    acc = ctx.accum_stats()

    # ---- the timed frames are distinct and correct: the last launch's first and last frame equal
    # their own single-frame render (rank 0, untimed)
    if not args.no_verify and rank == 0:
        last = target(F).download(t=False)
        n = W * H
        one = va.hip_buffer_rt(ctx, W, H)
        ok = True
        last_fn = first_timed + (launches - 1) * F
        for f in sorted({0, F - 1}):
            va.render(ctx, dev, one, basis, kern, None, frame_num=last_fn + f)
            single = one.download(t=False)
            ok &= all(np.array_equal(last[k][f * n:(f + 1) * n].view(np.uint8), single[k].view(np.uint8))
                      for k in ("color", "prim_id", "occ") if k in last)
        verify["timed_frames_match_single_frame_renders"] = bool(ok)
        if kernel == "ao" and F > 1:
            key = "occ" if "occ" in last else "color"
            verify["timed_frames_distinct"] = not np.array_equal(last[key][:n], last[key][(F - 1) * n:F * n])
        one.close()
    barrier()

    # ---- hip_sched::frame leg: one synchronous launch per frame (rank 0, N = 1) ---------------------
    single = None
    if world == 1 and args.single_frames > 0:
        rt_s = va.hip_buffer_rt(ctx, W, H)
        sched = va.hip_sched(ctx, async_frames=False)       # frame() returns when the frame is done
        sp = va.make_sched_params(va.pixel_sampler.uniform_type, cam, rt_s)
        k_ms, wall_ms, rays = [], [], []
        sched.frame(kern, sp, frame_num=next_frame[0])     # warm-up of this launch shape
        for i in range(args.single_frames):
            t1 = time.perf_counter()
            sched.frame(kern, sp, frame_num=next_frame[0] + 1 + i)
            wall_ms.append((time.perf_counter() - t1) * 1e3)
            st = ctx.last_frame_stats()
            k_ms.append(st["kernel_ms"])
            rays.append(st["rays"])
        rpf = statistics.median(rays)
        single = {"frames": args.single_frames, "kernel_ms_median": round(statistics.median(k_ms), 4),
                  "wall_ms_median": round(statistics.median(wall_ms), 4),
                  "mrays_kernel": round(rpf / statistics.median(k_ms) / 1e3, 3),
                  "mrays_wall": round(rpf / statistics.median(wall_ms) / 1e3, 3),
                  "path": "hip_sched::frame -> vrh_render + vrh_sync (one launch per frame)"}
        rt_s.close()

    # ---- hip_sched::frame with asynchronous issue (VRH_OPT_ASYNC_FRAMES, cuda_sched's model:
    # cuda_sched.inl:306-320 returns without a sync): --single-frames back-to-back frame() calls, one
    # final sync, into one shared target and into two alternating targets (rank 0, N = 1)
    single_async = None
    if world == 1 and not grouped and args.single_frames > 0:
        sched = va.hip_sched(ctx)                            # hip_sched's default: cuda_sched's issue model
        single_async = {"frames": args.single_frames,
                        "path": "hip_sched::frame x N, end_frame without sync, then one vrh_sync: frames "
                                "alternate between the context's two frame lanes (vrh.h VRH_OPT_ASYNC_FRAMES)"}
        ctx.set_option("async_frames", 1)
        try:
            for targets in (1, 2):
                rts_a = [va.hip_buffer_rt(ctx, W, H) for _ in range(targets)]
                for i in range(2):                       # warm-up: both lanes, scratch targets allocated
                    sched.frame(kern, va.make_sched_params(cam, rts_a[i % targets]), frame_num=next_frame[0])
                    next_frame[0] += 1
                ctx.sync()
                ctx.stats_reset()
                first = next_frame[0]
                t1 = time.perf_counter()
                for i in range(args.single_frames):
                    sched.frame(kern, va.make_sched_params(cam, rts_a[i % targets]), frame_num=first + i)
                ctx.sync()
                wall = time.perf_counter() - t1
                next_frame[0] += args.single_frames
                am = ctx.accum_stats()
                leg = {"targets": targets, "span_ms": round(am["span_ms"], 4), "wall_ms": round(wall * 1e3, 4),
                       "kernel_ms_per_frame_sum": round(am["kernel_ms_total"] / args.single_frames, 4),
                       "ms_per_frame": round(am["span_ms"] / args.single_frames, 4),
                       "mrays_span": round(am[rays_key] / am["span_ms"] / 1e3, 3),
                       "mrays_wall": round(am[rays_key] / wall / 1e6, 3)}
                if not args.no_verify and targets == 1:
                    # the shared target holds the last frame, equal to its own synchronous render
                    last = rts_a[0].download(t=False)
                    ctx.set_option("async_frames", 0)
                    one = va.hip_buffer_rt(ctx, W, H)
                    sched.frame(kern, va.make_sched_params(cam, one), frame_num=first + args.single_frames - 1)
                    ref1 = one.download(t=False)
                    one.close()
                    ctx.set_option("async_frames", 1)
                    verify["async_shared_target_holds_last_frame"] = all(
                        np.array_equal(last[k].view(np.uint8), ref1[k].view(np.uint8)) for k in last)
                for r in rts_a:
                    r.close()
                single_async["shared_target" if targets == 1 else "two_targets"] = leg
        finally:
            ctx.set_option("async_frames", 0)

    # ---- moving-camera leg (N = 1, untimed by the driver's clock): the timed launches' shape with
    # the eye orbiting --moving-camera degrees per frame, so no two frames of a launch share primary
    # rays (the timed frames share the scene camera, as the reference viewer's frames do at rest)
    moving = None
    if world == 1 and not grouped and args.moving_camera > 0:
        nl = 3
        bases = scenes.orbit_bases(args.scene, args.moving_camera, F * nl)
        rt_m = target(F)
        va.render_batch(ctx, dev, rt_m, bases[:F], kern, None, frame_num=next_frame[0])   # warm-up
        next_frame[0] += F
        sync()
        ctx.stats_reset()
        for k in range(nl):
            va.render_batch(ctx, dev, rt_m, bases[k * F:(k + 1) * F], kern, None, frame_num=next_frame[0])
            next_frame[0] += F
        sync()
        am = ctx.accum_stats()
        moving = {"degrees_per_frame": args.moving_camera, "frames_per_launch": F, "launches": nl,
                  "kernel_ms_per_frame": round(am["kernel_ms_total"] / (nl * F), 4),
                  "mrays_kernel": round(am[rays_key] / am["kernel_ms_total"] / 1e3, 3),
                  "what": "same launches as the timed region, eye orbiting the scene centre per frame "
                          "(scenes.orbit_bases); kernel time from hipEvents"}

    # ---- aggregate over ranks -------------------------------------------------------------------
    local_vals = torch.tensor([elapsed, float(acc[rays_key]), acc["kernel_ms_total"], float(acc["timed_frames"])],
                              dtype=torch.float64, device="cuda")
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
        s_prim = TRI_BYTES if args.scene.startswith("hf") or args.scene == "cornell12" else SPHERE_BYTES
        n_box, n_prim, n_rays = float(cstats["box_tests"]), float(cstats["prim_tests"]), float(cstats["rays"])
        bytes_frame = NODE_BYTES * n_box + (s_prim + INDEX_BYTES) * n_prim + OUT_BYTES_PRIMARY * W * H
        bytes_per_ray = bytes_frame / n_rays
        # the dominant kernel: rank 0's traversal launches of the timed region (F frames each)
        k_ms_mean = float(local_vals[2]) / max(float(local_vals[3]), 1.0)
        rays_launch = float(acc[rays_key]) / max(float(acc["timed_frames"]), 1.0)
        frame_share = rays_launch / n_rays                      # frames per launch on this rank (N > 1: a shard)
        roof = load_json(os.path.join(ROOT, "profiles", "l1_roof.json"))
        pieces_launch = float(cstats["l1_requests"]) * frame_share    # counting variant: distinct 16-B pieces
        peak = roof.get("peak_gbs") if roof else None
        hbm_alg = bytes_per_ray * rays_launch / (k_ms_mean * 1e-3) / 1e9
        # PMC of this exact configuration (tools/session.sh pmc:<cfg> + tools/pmc_bench.py): HBM bytes per
        # launch (`traffic`), the L1 requests the hardware counted and how busy the TD unit was
        # one committed pass per frames-per-launch value (the driver's --steps decides F)
        # (most specific first: scene + kernel, scene, the C3 default)
        pmc_name = next((n for n in (f"pmc_traffic_F{F}_{args.scene}_{kernel}.json", f"pmc_traffic_F{F}_{args.scene}.json")
                         if os.path.exists(os.path.join(ROOT, "profiles", n))), f"pmc_traffic_F{F}.json")
        pmc = load_json(os.path.join(ROOT, "profiles", pmc_name)) or {}
        traffic, pmc_info = None, None
        from visionaray_amd.buildinfo import kernel_source_sha256
        pmc_build_ok = pmc.get("kernel_source_sha256") == kernel_source_sha256()
        if (pmc.get("scene") == args.scene and pmc.get("kernel") == kernel and not grouped
                and pmc.get("frames_per_launch") == F and pmc_build_ok):
            traffic = pmc.get("hbm_bytes_per_launch")
            if pmc.get("l1_requests_per_launch"):
                pmc_info = {"l1_requests_per_launch": pmc["l1_requests_per_launch"],
                            "td_busy_frac": round(pmc["td_busy_frac"], 4),
                            "source": f"profiles/{pmc_name}: " + pmc.get("command", "")}
                # the load-count model: time follows the wave-level vector loads at a
                # near-constant TD cost per load -- SQ_INSTS_VMEM_RD per ray and TD busy cycles per load
                cpl = pmc.get("counters_per_launch") or {}
                if cpl.get("SQ_INSTS_VMEM_RD") and cpl.get("TD_TD_BUSY_sum"):
                    loads = cpl["SQ_INSTS_VMEM_RD"]
                    pmc_info["wave_loads_per_launch"] = round(loads)
                    pmc_info["wave_loads_per_frame"] = round(loads / F)
                    pmc_info["wave_loads_per_ray"] = round(loads / rays_launch, 4)
                    pmc_info["td_cycles_per_load"] = round(cpl["TD_TD_BUSY_sum"] / loads, 3)
                    pmc_info["l1_requests_per_load"] = round(pmc["l1_requests_per_launch"] / loads, 3)
        # achieved: the hardware-counted L1 requests (TCP_TOTAL_CACHE_ACCESSES) of a committed PMC pass
        # of this exact configuration, over the live hipEvent time; without one it is not reported
        achieved = (pmc_info["l1_requests_per_launch"] * L1_REQ_BYTES / (k_ms_mean * 1e-3) / 1e9) if pmc_info else None
        # the roof of the kernel's own access shape: the fastest microbenchmark mode whose loads are
        # at least as merged as the kernel's (TCP accesses per wave-level load <= 1.25 x the kernel's,
        # PMC) -- for ~17.6 that is "quad-bcast" (4 lanes per address, 16 accesses per load); the
        # max-rate `peak` mode is per-lane gathers at 64 accesses per load
        shape = None
        if roof and pmc and pmc.get("l1_requests_per_vmem_load") and pmc_info:
            apl = pmc["l1_requests_per_vmem_load"]
            cands = {k: v for k, v in roof["modes"].items() if v["tcp_accesses_per_load"] <= 1.25 * apl} or roof["modes"]
            name, m = max(cands.items(), key=lambda kv: kv[1]["requests_per_s"])
            sp = m["requests_per_s"] * L1_REQ_BYTES / 1e9
            shape = {"mode": name, "accesses_per_load": round(m["tcp_accesses_per_load"], 2),
                     "kernel_accesses_per_load": round(apl, 2), "peak": round(sp, 1),
                     "frac": round(achieved / sp, 4)}
        user_leg = None
        if world == 1 and args.scene == "hf1M" and kernel == "ao" and not args.no_user_kernel and not grouped:
            user_leg = user_kernel_leg(W, H, n_rays)
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
            "data": "synthetic (SURVEY.md Appendix A procedural scene, deterministic; frame numbers 1.. give distinct AO samples)",
            "config": {
                "workload": f"{args.scene} {W}x{H} 1 spp primary" + (" + 8 AO any-hit rays/hit (r=0.1)" if kernel == "ao" else ""),
                "scene": args.scene, "primitives": int(len(prims)), "bvh_nodes": int(len(host.nodes)),
                "width": W, "height": H, "ao_samples": 8 if kernel == "ao" else 0,
                "rays_per_frame": int(n_rays),
                "parallelism": f"image-tile shard x{world}" + (f" ({args.shards} shards)" if args.shards else "")
                               + (" + RCCL gather (libvrh render group)" if grouped else ""),
                "frames_per_launch": F, "launches": launches,
                "frame_numbers": [first_timed, first_timed + args.steps - 1],
            },
            "roofline": {
                "bound": "vmem-l1", "unit": "GB/s",
                "achieved": round(achieved, 1) if achieved else None, "peak": peak,
                "frac": round(achieved / peak, 4) if (peak and achieved) else None,
                "own_shape": shape,
                "traffic": traffic,
                "what": "vector-L1 requests (TCP accesses: distinct 16-B pieces per wave-level load/store) x 16 B of "
                        "the traversal launch over its hipEvent time; peak = the request rate of per-lane dependent "
                        "64-B record gathers on tools/micro/l1_roof.hip (profiles/l1_roof.json)",
                "kernel": "render_unified_kernel (traversal, frames in flight)" if F > 1 else "render_unified_kernel",
                "kernel_ms_mean": round(k_ms_mean, 4), "frames_per_launch": F,
                "kernel_ms_per_frame": round(k_ms_mean / F, 4),
                "roof_source": roof.get("source") if roof else None,
                "requests_source": ("pmc (TCP_TOTAL_CACHE_ACCESSES of the committed pass)" if pmc_info
                                    else "the committed PMC pass is of another kernel build (kernel_source_sha256 "
                                         "differs): achieved / frac / traffic not reported" if pmc and not pmc_build_ok
                                    else "no PMC pass of this configuration committed: achieved / frac not reported"),
                "pmc": pmc_info,
                # the counting variant's access-shape statistics of one frame (diagnostic; they count
                # distinct 16-B pieces and 128-B lines per wave-level access, not TCP accesses)
                "counted": {"distinct_16B_pieces_per_launch": round(pieces_launch),
                            "distinct_16B_pieces_per_ray": round(float(cstats["l1_requests"]) / n_rays, 3),
                            "vmem_instrs_per_ray": round(float(cstats["vmem_instrs"]) / n_rays, 3),
                            "lines128_per_vmem_instr": round(float(cstats["l1_lines"]) / max(float(cstats["vmem_instrs"]), 1.0), 3),
                            # the vector L1's 4-lane merging: accesses as the lanes sit (the model of
                            # TCP_TOTAL_CACHE_ACCESSES) and if lanes wanting one piece sat together
                            "group4_accesses_per_launch": round(float(cstats.get("l1_group_accesses", 0)) * frame_share),
                            "ideal_group_accesses_per_launch": round(float(cstats.get("l1_ideal_accesses", 0)) * frame_share)},
                "hbm_algorithmic": {
                    "bytes_per_ray": round(bytes_per_ray, 1), "box_tests_per_ray": round(n_box / n_rays, 3),
                    "prim_tests_per_ray": round(n_prim / n_rays, 3), "achieved_gbs": round(hbm_alg, 1),
                    "frac_of_8tbs": round(hbm_alg / HBM_PEAK_GBS, 4),
                    "note": "SURVEY.md §8d algorithmic bytes; the scene lives in L2 / Infinity Cache, so this is not "
                            "HBM traffic (that is `traffic`)"},
            },
            "single_frame": single,
            "single_frame_mrays": single["mrays_kernel"] if single else None,
            "single_frame_async": single_async,
            "single_frame_async_mrays": single_async["shared_target"]["mrays_span"] if single_async else None,
            "moving_camera": moving,
            "moving_camera_mrays": moving["mrays_kernel"] if moving else None,
            "cpu_baseline": cpu,
            "user_kernel": user_leg,
            "user_kernel_mrays": user_leg.get("mrays") if user_leg else None,
            "user_kernel_deferred_mrays": (user_leg.get("deferred") or {}).get("mrays") if user_leg else None,
            "host_build_s": round(build_s, 3),
            "settle": settle,
            "verify": verify,
        }
        print(json.dumps(line), file=json_out, flush=True)

    if group is not None:
        barrier()
        group.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except BaseException:
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            # a failed rank leaves at once, without the barrier or the group's teardown: the other ranks'
            # deadlines (GROUP_TIMEOUT_MS) end them with an error instead of a hang
            import traceback
            traceback.print_exc()
            sys.stderr.flush()
            os._exit(3)
        raise
