"""Regenerate tests/golden/ from the reference itself (oracle/_ref/vsnray_ref).

Run in the build container (needs /root/reference to build the harness):

    make -C oracle ref && python tests/golden/make_golden.py            (everything)
    python tests/golden/make_golden.py --shade                          (shading + multi-hit cases)
    python tests/golden/make_golden.py --multi                          (only the multi-hit cases)
    python tests/golden/make_golden.py --sah                            (only the sah_cost values)
    python tests/golden/make_golden.py --whitted                        (only the whitted cases)
    python tests/golden/make_golden.py --mask                           (only the mask-intersector cases)
    python tests/golden/make_golden.py --frames                         (only the frame-number cases)
    python tests/golden/make_golden.py --list                           (only the BVH-list + scissor cases)
    python tests/golden/make_golden.py --heart                          (only the procedural-heart cases)
    python tests/golden/make_golden.py --sampler                        (only the pixel-sampler cases)
    python tests/golden/make_golden.py --rsampler                       (only the random_sampler AO cases)

For every case the reference harness renders a full simple_sched<basic_ray<float>> frame
(primary closest_hit + the Appendix-A AO kernel for triangle scenes) and this script stores:
  * golden.json            : per case counts, BVH/pixel FNV-1a-64 hashes (bytes, little endian),
                             camera basis bits, tree depth;
  * <case>.npz             : small cases -> every pixel (prim_id, t, occ, colour) + the BVH;
                             large cases -> a fixed sample of 4096 pixels.
The fixtures are data (inputs are the deterministic Appendix-A generators, outputs are what the
reference computed); no reference source is stored.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref", "vsnray_ref")
REF_CLANG = os.path.join(ROOT, "oracle", "_ref", "vsnray_ref_clang")    # the harness built by clang++ (rsampler)

# (case name, scene, W, H, full dump?)
CASES = [
    ("cornell12", "cornell12", 512, 512, True),
    ("hf64_160x90", "hf64", 160, 90, True),
    ("hf200_320x180", "hf200", 320, 180, True),
    ("sph5000_256x144", "sph5000", 256, 144, True),
    ("hf1M", "hf1M", 1920, 1080, False),
    ("sph1M", "sph1M", 1920, 1080, False),
    ("hf10M", "hf10M", 1920, 1080, False),
]


# simple::kernel shading cases (reference harness "shade" mode): (case, scene, W, H, binding, full dump?)
SHADE_CASES = [
    ("shade_cornell12_face", "cornell12", 128, 128, "face", True),
    ("shade_cornell12_vertex", "cornell12", 128, 128, "vertex", True),
    ("shade_hf64_face", "hf64", 160, 90, "face", True),
    ("shade_hf64_vertex", "hf64", 160, 90, "vertex", True),
    ("shade_hf1M_vertex", "hf1M", 1920, 1080, "vertex", False),
]


# multi_hit<16> cases (harness "multi" mode): hit lists + the multi_hit example's colour
MULTI_CASES = [
    ("multi_cornell12_face", "cornell12", 128, 128, "face"),
    ("multi_hfstack32x24_face", "hfstack32x24", 160, 90, "face"),
    ("multi_hfstack32x24_vertex", "hfstack32x24", 160, 90, "vertex"),
]


# whitted::kernel cases (harness "whitted" mode, whitted_spec): name, scene, W, H, binding,
# num_bounces, epsilon, full frame?
WHITTED_CASES = [
    ("whitted_cornell12_face", "cornell12", 128, 128, "face", 4, "0.001", True),
    ("whitted_cornell12_vertex", "cornell12", 128, 128, "vertex", 6, "0.0005", True),
    ("whitted_hfstack32x24_face", "hfstack32x24", 160, 90, "face", 10, "0.0001", True),
    ("whitted_hf64_vertex", "hf64", 160, 90, "vertex", 2, "0.01", True),
    ("whitted_hf1M_face", "hf1M", 1920, 1080, "face", 4, "0.001", False),
]


# mask intersector cases (harness "mask" mode): the intersector example's mask_intersector with a
# heart-shaped byte mask over planar (x, z) texture coordinates: name, scene, W, H, mask size
MASK_CASES = [
    ("mask_hf200_320x180", "hf200", 320, 180, 128),
    ("mask_hf64_160x90", "hf64", 160, 90, 37),
]


# procedural-heart cases (harness "heart" mode): primary closest hit with the intersector example's
# procedural cut-out over planar (x, z) texture coordinates: name, scene, W, H
HEART_CASES = [
    ("heart_hf64_160x90", "hf64", 160, 90),
    ("heart_hf200_320x180", "hf200", 320, 180),
]


# frame-number cases (harness "golden" mode with a frame number: the AO sampler of frame n, vrh.h
# vrh_render): name, scene, W, H, frame number, full frame?
FRAME_CASES = [
    ("frame7_hf64_160x90", "hf64", 160, 90, 7, True),
    ("frame1_hf200_320x180", "hf200", 320, 180, 1, True),
    ("frame3_hf1M", "hf1M", 1920, 1080, 3, False),
]


# BVH-ref list + scissor cases (harness "list" mode: the scene's triangles split by prim_id parity
# into two BVHs, closest_hit / any_hit over the list, tiled_sched with a scissor box): name, scene,
# W, H, scissor (x0, y0, x1, y1: pixels x0 <= x < x1, y0 <= y < y1), frame number
LIST_CASES = [
    ("list_hf64_160x90", "hf64", 160, 90, (17, 9, 141, 77), 3),
    ("list_hf200_320x180", "hf200", 320, 180, (40, 30, 300, 150), 0),
    ("list_cornell12_128", "cornell12", 128, 128, (5, 0, 128, 100), 11),
]


# sah_cost (detail/bvh/statistics.h) of the reference's own trees
SAH_SCENES = ["cornell12", "hf64", "hf200", "sph5000", "hf1M", "sph1M"]


def fnv1a(a):
    """FNV-1a 64 over the little-endian bytes (computed by the oracle's C helper for speed)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O  # noqa: E402
    return O.fnv1a(np.ascontiguousarray(a).view(np.uint8).reshape(-1))


def shade_cases(out, rng):
    for case, scene, W, H, binding, full in SHADE_CASES:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF, "shade", scene, d, binding, str(W), str(H)], check=True, capture_output=True,
                               text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            color = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            rec = {"scene": scene, "W": W, "H": H, "binding": binding, "color_hash": fnv1a(color)}
            assert rec["color_hash"] == info["color_hash"]
            if full:
                np.savez_compressed(os.path.join(HERE, case + ".npz"), color=color)
            else:
                pix = np.sort(rng.choice(W * H, 4096, replace=False)).astype(np.uint32)
                np.savez_compressed(os.path.join(HERE, case + ".npz"), pixels=pix, color=color[pix])
            out[case] = rec
            print(case, rec["color_hash"], flush=True)


def multi_cases(out):
    for case, scene, W, H, binding in MULTI_CASES:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF, "multi", scene, d, binding, str(W), str(H)], check=True, capture_output=True,
                               text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            color = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            pid = np.fromfile(os.path.join(d, "mh_prim_id.bin"), np.uint32).reshape(W * H, -1)
            t = np.fromfile(os.path.join(d, "mh_t.bin"), np.float32).reshape(W * H, -1)
            rec = {"scene": scene, "W": W, "H": H, "binding": binding, "max_hits": info["max_hits"],
                   "hits": info["hits"], "color_hash": fnv1a(color), "mh_primid_hash": fnv1a(pid),
                   "mh_t_hash": fnv1a(t)}
            np.savez_compressed(os.path.join(HERE, case + ".npz"), color=color, mh_prim_id=pid, mh_t=t)
            out[case] = rec
            print(case, rec["hits"], rec["color_hash"], flush=True)


def whitted_cases(out, rng):
    for case, scene, W, H, binding, bounces, eps, full in WHITTED_CASES:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF, "whitted", scene, d, binding, str(W), str(H), str(bounces), eps], check=True,
                               capture_output=True, text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            color = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            rec = {"scene": scene, "W": W, "H": H, "binding": binding, "bounces": bounces, "eps": float(eps),
                   "color_hash": fnv1a(color)}
            assert rec["color_hash"] == info["color_hash"]
            if full:
                np.savez_compressed(os.path.join(HERE, case + ".npz"), color=color)
            else:
                pix = np.sort(rng.choice(W * H, 4096, replace=False)).astype(np.uint32)
                np.savez_compressed(os.path.join(HERE, case + ".npz"), pixels=pix, color=color[pix])
            out[case] = rec
            print(case, rec["color_hash"], flush=True)


def mask_cases(out):
    sys.path.insert(0, ROOT)
    from visionaray_amd import scenes  # noqa: E402  (the heart mask generator)
    for case, scene, W, H, n in MASK_CASES:
        mask = scenes.heart_mask(n)
        with tempfile.TemporaryDirectory() as d:
            mpath = os.path.join(d, "mask.bin")
            mask.tofile(mpath)
            r = subprocess.run([REF, "mask", scene, d, mpath, str(n), str(n), str(W), str(H)], check=True,
                               capture_output=True, text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            pid = np.fromfile(os.path.join(d, "prim_id.bin"), np.uint32)
            t = np.fromfile(os.path.join(d, "t.bin"), np.float32)
            occ = np.fromfile(os.path.join(d, "occ.bin"), np.uint8)
            color = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            tc = np.fromfile(os.path.join(d, "tex_coords.bin"), np.float32).reshape(-1, 2)
            rec = {"scene": scene, "W": W, "H": H, "mask_size": n, "hits": info["hits"], "ao_rays": info["ao_rays"],
                   "ao_occluded": info["ao_occluded"], "primid_hash": fnv1a(pid), "t_hash": fnv1a(t),
                   "occ_hash": fnv1a(occ), "color_hash": fnv1a(color), "tex_coords_hash": fnv1a(tc)}
            np.savez_compressed(os.path.join(HERE, case + ".npz"), prim_id=pid, t=t, occ=occ, color=color, mask=mask)
            out[case] = rec
            print(case, rec["hits"], rec["ao_occluded"], flush=True)


def heart_cases(out):
    for case, scene, W, H in HEART_CASES:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF, "heart", scene, d, str(W), str(H)], check=True, capture_output=True, text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            pid = np.fromfile(os.path.join(d, "prim_id.bin"), np.uint32)
            t = np.fromfile(os.path.join(d, "t.bin"), np.float32)
            rec = {"scene": scene, "W": W, "H": H, "hits": info["hits"], "primid_hash": fnv1a(pid), "t_hash": fnv1a(t)}
            np.savez_compressed(os.path.join(HERE, case + ".npz"), prim_id=pid, t=t)
            out[case] = rec
            print(case, rec["hits"], flush=True)


def frame_cases(out, rng):
    for case, scene, W, H, frame, full in FRAME_CASES:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF, "golden", scene, d, str(W), str(H), str(frame)], check=True, capture_output=True,
                               text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            pid = np.fromfile(os.path.join(d, "prim_id.bin"), np.uint32)
            t = np.fromfile(os.path.join(d, "t.bin"), np.float32)
            occ = np.fromfile(os.path.join(d, "occ.bin"), np.uint8)
            color = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            rec = {"scene": scene, "W": W, "H": H, "frame": frame, "hits": info["hits"], "ao_rays": info["ao_rays"],
                   "ao_occluded": info["ao_occluded"], "primid_hash": fnv1a(pid), "t_hash": fnv1a(t),
                   "occ_hash": fnv1a(occ), "color_hash": fnv1a(color)}
            if full:
                np.savez_compressed(os.path.join(HERE, case + ".npz"), prim_id=pid, t=t, occ=occ, color=color)
            else:
                pix = np.sort(rng.choice(W * H, 4096, replace=False)).astype(np.uint32)
                np.savez_compressed(os.path.join(HERE, case + ".npz"), pixels=pix, prim_id=pid[pix], t=t[pix],
                                    occ=occ[pix], color=color[pix])
            out[case] = rec
            print(case, rec["hits"], rec["ao_occluded"], rec["occ_hash"], flush=True)


def list_cases(out):
    for case, scene, W, H, sb, frame in LIST_CASES:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF, "list", scene, d, str(W), str(H)] + [str(v) for v in sb] + [str(frame)],
                               check=True, capture_output=True, text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            arr = {k: np.fromfile(os.path.join(d, k + ".bin"), dt) for k, dt in
                   (("prim_id", np.uint32), ("t", np.float32), ("occ", np.uint8), ("leaf_pos", np.uint32))}
            arr["color"] = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            for k in (0, 1):
                arr[f"bvh{k}_nodes"] = np.fromfile(os.path.join(d, f"bvh{k}_nodes.bin"), np.uint32)
                arr[f"bvh{k}_indices"] = np.fromfile(os.path.join(d, f"bvh{k}_indices.bin"), np.uint32)
                arr[f"bvh{k}_prims"] = np.fromfile(os.path.join(d, f"bvh{k}_prims.bin"), np.uint8)
            rec = {"scene": scene, "W": W, "H": H, "scissor": list(sb), "frame": frame, "hits": info["hits"],
                   "ao_rays": info["ao_rays"], "ao_occluded": info["ao_occluded"],
                   "primid_hash": fnv1a(arr["prim_id"]), "t_hash": fnv1a(arr["t"]), "occ_hash": fnv1a(arr["occ"]),
                   "color_hash": fnv1a(arr["color"])}
            for k in ("primid_hash", "t_hash", "color_hash"):
                assert rec[k] == info[k], (case, k, rec[k], info[k])
            np.savez_compressed(os.path.join(HERE, case + ".npz"), **arr)
            out[case] = rec
            print(case, rec["hits"], rec["ao_occluded"], flush=True)


# (case, scene, kernel, sampler, frame, W, H): the reference's pixel samplers (harness `sampler` mode)
SAMPLER_CASES = [(f"sampler_{k}_hf64_ao", "hf64", "ao", k, 3, 160, 90)
                 for k in ("uniform", "jittered", "jittered_blend", "ssaa2", "ssaa4", "ssaa8")] + [
    ("sampler_ssaa8_sph5000_primary", "sph5000", "primary", "ssaa8", 2, 128, 72),
    ("sampler_jittered_blend_sph5000_primary", "sph5000", "primary", "jittered_blend", 2, 128, 72),
    ("sampler_jittered_blend_hf200_ao", "hf200", "ao", "jittered_blend", 3, 320, 180),
    ("sampler_ssaa4_hf200_ao", "hf200", "ao", "ssaa4", 3, 320, 180),
    # the camera as view / projection matrices (sched_params with MT), alone and with samplers
    ("matrix_uniform_hf64_ao", "hf64", "ao", "uniform+matrix", 3, 160, 90),
    ("matrix_ssaa4_hf64_ao", "hf64", "ao", "ssaa4+matrix", 3, 160, 90),
    ("matrix_jittered_blend_sph5000_primary", "sph5000", "primary", "jittered_blend+matrix", 2, 128, 72),
    ("matrix_uniform_hf200_ao", "hf200", "ao", "uniform+matrix", 0, 320, 180),
]


def sampler_cases(out):
    for case, scene, kernel, kind, frame, W, H in SAMPLER_CASES:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF, "sampler", scene, d, kind, kernel, str(frame), str(W), str(H)], check=True,
                               capture_output=True, text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            pid = np.fromfile(os.path.join(d, "prim_id.bin"), np.uint32)
            t = np.fromfile(os.path.join(d, "t.bin"), np.float32)
            color = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            sampler, _, cam = kind.partition("+")
            rec = {"scene": scene, "kernel": kernel, "sampler": sampler, "camera": cam or "pinhole", "frame": frame,
                   "W": W, "H": H, "primid_hash": fnv1a(pid), "t_hash": fnv1a(t), "color_hash": fnv1a(color)}
            assert rec["primid_hash"] == info["primid_hash"] and rec["color_hash"] == info["color_hash"], case
            arrays = {"prim_id": pid, "t": t, "color": color}
            if cam == "matrix":
                arrays["view"] = np.fromfile(os.path.join(d, "view.bin"), np.float32)
                arrays["proj"] = np.fromfile(os.path.join(d, "proj.bin"), np.float32)
            np.savez_compressed(os.path.join(HERE, case + ".npz"), **arrays)
            out[case] = rec
            print(case, rec["color_hash"], flush=True)


# (case, scene, W, H, frame): the AO example's kernel verbatim with random_sampler<float> seeded per pixel
# as hip_sched seeds it (harness `rsampler` mode, built by clang++): draws 0, 1, 2, 15 of every pixel's
# sampler, the closest-hit t, the AO colour.  Stored: hashes over the whole frame, the occluded-sample
# count per pixel (255 = miss), and 4096 sampled pixels' draws and t.
RSAMPLER_CASES = [
    ("rs_hf64_160x90_f0", "hf64", 160, 90, 0),
    ("rs_hf200_320x180_f3", "hf200", 320, 180, 3),
    ("rs_hf1M_f1", "hf1M", 1920, 1080, 1),
]


def rsampler_cases(out):
    rng = np.random.default_rng(97531)
    for case, scene, W, H, frame in RSAMPLER_CASES:
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF_CLANG, "rsampler", scene, d, str(W), str(H), str(frame)], check=True,
                               capture_output=True, text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            draws = np.fromfile(os.path.join(d, "draws.bin"), np.float32).reshape(-1, 4)
            t = np.fromfile(os.path.join(d, "t.bin"), np.float32)
            color = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            hit = t >= 0.0
            k = np.where(hit, np.rint((1.0 - color[:, 0]) * 8.0), 255).astype(np.uint8)
            rec = {"scene": scene, "W": W, "H": H, "frame": frame, "samples": 8, "hits": int(hit.sum()),
                   "draws_hash": fnv1a(draws), "t_hash": fnv1a(t), "color_hash": fnv1a(color),
                   "occluded_samples": int(k[hit].astype(np.int64).sum())}
            assert rec["draws_hash"] == info["draws_hash"] and rec["color_hash"] == info["color_hash"], case
            pix = np.sort(rng.choice(W * H, 4096, replace=False)).astype(np.uint32)
            np.savez_compressed(os.path.join(HERE, case + ".npz"), ao_count=k, pixels=pix, draws=draws[pix], t=t[pix])
            out[case] = rec
            print(case, rec["hits"], rec["occluded_samples"], rec["draws_hash"], flush=True)


def sah_cases(out):
    rec = {}
    for scene in SAH_SCENES:
        r = subprocess.run([REF, "sah", scene], check=True, capture_output=True, text=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        rec[scene] = info["sah_cost_bits"]
        print("sah", scene, info["sah_cost"], flush=True)
    out["sah_cost_bits"] = rec


def main():
    if not os.path.exists(REF):
        sys.exit("build the reference harness first: make -C oracle ref")
    only_shade = any(f in sys.argv for f in ("--shade", "--multi", "--sah", "--whitted", "--mask", "--frames", "--list",
                                                "--heart", "--sampler", "--rsampler"))
    path = os.path.join(HERE, "golden.json")
    out = json.load(open(path)) if only_shade else {}
    rng = np.random.default_rng(12345)
    for case, scene, W, H, full in ([] if only_shade else CASES):
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([REF, "golden", scene, d, str(W), str(H)], check=True, capture_output=True, text=True)
            info = json.loads(r.stdout.strip().splitlines()[-1])
            pid = np.fromfile(os.path.join(d, "prim_id.bin"), np.uint32)
            t = np.fromfile(os.path.join(d, "t.bin"), np.float32)
            color = np.fromfile(os.path.join(d, "color.bin"), np.float32).reshape(-1, 4)
            occp = os.path.join(d, "occ.bin")
            occ = np.fromfile(occp, np.uint8) if os.path.exists(occp) else np.zeros(W * H, np.uint8)
            nodes = np.fromfile(os.path.join(d, "nodes.bin"), np.uint32)
            idx = np.fromfile(os.path.join(d, "indices.bin"), np.uint32)
            rec = {
                "scene": scene, "W": W, "H": H, "prims": info["prims"], "nodes": info["nodes"],
                "max_depth": info["max_depth"], "hits": info["hits"], "ao_rays": info["ao_rays"],
                "ao_occluded": info["ao_occluded"],
                "bvh_hash": fnv1a(nodes), "idx_hash": fnv1a(idx),
                "primid_hash": fnv1a(pid), "t_hash": fnv1a(t), "occ_hash": fnv1a(occ), "color_hash": fnv1a(color),
                "cam_u": info["cam_u"], "cam_v": info["cam_v"], "cam_w": info["cam_w"],
            }
            if full:
                np.savez_compressed(os.path.join(HERE, case + ".npz"), prim_id=pid, t=t, occ=occ, color=color,
                                    nodes=nodes, indices=idx)
            else:
                pix = np.sort(rng.choice(W * H, 4096, replace=False)).astype(np.uint32)
                np.savez_compressed(os.path.join(HERE, case + ".npz"), pixels=pix, prim_id=pid[pix], t=t[pix],
                                    occ=occ[pix], color=color[pix])
            out[case] = rec
            print(case, rec["hits"], rec["ao_occluded"], rec["primid_hash"], flush=True)
    if "--heart" in sys.argv:
        heart_cases(out)
    elif "--rsampler" in sys.argv:
        rsampler_cases(out)
    elif "--sampler" in sys.argv:
        sampler_cases(out)
    elif "--frames" in sys.argv:
        frame_cases(out, np.random.default_rng(2468))
    elif "--list" in sys.argv:
        list_cases(out)
    elif "--mask" in sys.argv:
        mask_cases(out)
    elif "--whitted" in sys.argv:
        whitted_cases(out, np.random.default_rng(777))
    elif "--sah" in sys.argv:
        sah_cases(out)
    else:
        if "--multi" not in sys.argv:
            shade_cases(out, np.random.default_rng(54321))
        multi_cases(out)
        sah_cases(out)
        whitted_cases(out, np.random.default_rng(777))
        mask_cases(out)
        frame_cases(out, np.random.default_rng(2468))
        list_cases(out)
        sampler_cases(out)
        rsampler_cases(out)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
