"""CPU, world_size 2 and 3 over gloo: the protocol of libvrh's render groups (vrh_render_sharded),
driven through libvrh's own host exports of the plan (visionaray_amd/multigpu.py) -- shard ownership s -> rank s % N, packed shard buffers
of several frames on the wire as [prim ids | AO masks] (or one colour code byte per pixel), point-to-point sends / receives paired in
plan order, the root's un-interleave and colour re-derivation, the ray-count sum and max-over-ranks
timing of bench.py -- reproduces the single-process frames bit for bit, including S > N and S < N.
The per-rank renderer is the oracle restricted to the shard's rows; on the GPU box the same
protocol runs inside libvrh over RCCL (tests/test_gpu_group.py: a one-rank group with S shards)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from visionaray_amd import _capi, multigpu

SCENE, W, H, FRAMES, FRAME0 = "hf64", 160, 90, 2, 4
BG = (0.1, 0.2, 0.3, 1.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


FIELDS_IDS = _capi.VRH_RT_COLOR | _capi.VRH_RT_PRIM_ID | _capi.VRH_RT_OCC
FIELDS_ALL = FIELDS_IDS | _capi.VRH_RT_T
FIELDS_COLOR = _capi.VRH_RT_COLOR


def _worker(rank, world, shards, port, outdir, fields):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        sc = O.make_scene(SCENE)
        cam = O.scene_camera(SCENE, W, H)
        wire = multigpu.wire_layout(fields, W, H, FRAMES, shards, bg=BG)
        rm, nbytes = wire.rows, wire.shard_bytes
        sends, recvs = multigpu.exchange_plan(rank, world, shards)
        rays = 0
        bufs = []
        for s, _ in sends:                           # render every owned shard, packed
            buf = np.zeros(nbytes, np.uint8)
            pid = np.full((FRAMES, rm * W), 0xFFFFFFFF, np.uint32)
            occ = np.zeros((FRAMES, rm * W), np.uint8)
            t = np.zeros((FRAMES, rm * W), np.float32)
            for f in range(FRAMES):
                for lr, y in enumerate(multigpu.packed_rows(H, s, shards)):
                    if y < 0:
                        continue
                    out = O.render(sc, cam, mode=O.VO_MODE_AO, rows=(int(y), int(y) + 1), threads=1,
                                   frame_num=FRAME0 + f)
                    pid[f, lr * W:(lr + 1) * W] = out["prim_id"][y * W:(y + 1) * W]
                    occ[f, lr * W:(lr + 1) * W] = out["occ"][y * W:(y + 1) * W]
                    t[f, lr * W:(lr + 1) * W] = out["t"][y * W:(y + 1) * W]
                    rays += out["rays"]
            # the fields the library's layout puts on the wire, where it puts them
            if wire.prim_id != _capi.VRH_WIRE_ABSENT:
                multigpu.field(buf, wire, "prim_id", FRAMES, W, np.uint32)[:] = pid
            if wire.occ != _capi.VRH_WIRE_ABSENT:
                multigpu.field(buf, wire, "occ", FRAMES, W, np.uint8)[:] = occ
            if wire.t != _capi.VRH_WIRE_ABSENT:
                multigpu.field(buf, wire, "t", FRAMES, W, np.float32)[:] = t
            if wire.code != _capi.VRH_WIRE_ABSENT:
                multigpu.field(buf, wire, "code", FRAMES, W, np.uint8)[:] = \
                    multigpu.pack_code(pid.reshape(-1), occ.reshape(-1)).reshape(FRAMES, -1)
            bufs.append(torch.from_numpy(buf))
        # the exchange: sends to the root in plan order; the root receives shard s from s % N
        gathered = np.zeros((shards, nbytes), np.uint8) if rank == 0 else None
        reqs = [dist.isend(b, dst=0) for b, (s, peer) in zip(bufs, sends) if rank != 0]
        if rank == 0:
            mine = dict(zip([s for s, _ in sends], bufs))
            for s, peer in recvs:
                if peer == 0:
                    gathered[s] = mine[s].numpy()
                else:
                    tt = torch.empty(nbytes, dtype=torch.uint8)
                    dist.recv(tt, src=peer)
                    gathered[s] = tt.numpy()
        for r in reqs:
            r.wait()
        stats = torch.tensor([float(rank + 1), float(rays)], dtype=torch.float64)
        mx, sm = stats.clone(), stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        if rank == 0:
            for f in range(FRAMES):
                out = multigpu.unshard(gathered, wire, fields, W, H, shards, f, bg=BG)
                for key, a in out.items():
                    np.save(os.path.join(outdir, f"{key}{f}.npy"), a)
            np.save(os.path.join(outdir, "stats.npy"), np.array([mx[0].item(), sm[1].item()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shards,fields", [(2, 2, FIELDS_IDS), (3, 3, FIELDS_IDS), (2, 5, FIELDS_ALL),
                                                 (2, 3, FIELDS_COLOR), (3, 2, FIELDS_IDS)])
def test_sharded_exchange_equals_single_frames(tmp_path, oracle_mod, world, shards, fields):
    """FIELDS_COLOR: a colour-only target, one code byte per pixel on the wire (bench.py's N > 1
    default). (3, 2): fewer shards than ranks -- rank 2 renders and sends nothing."""
    O = oracle_mod
    mp.start_processes(_worker, args=(world, shards, _free_port(), str(tmp_path), fields), nprocs=world, join=True,
                       start_method="spawn")
    st = np.load(tmp_path / "stats.npy")
    rays = 0
    for f in range(FRAMES):
        full = O.render(O.make_scene(SCENE), O.scene_camera(SCENE, W, H), mode=O.VO_MODE_AO, frame_num=FRAME0 + f)
        rays += full["rays"]
        if fields & _capi.VRH_RT_PRIM_ID:
            assert np.array_equal(np.load(tmp_path / f"prim_id{f}.npy"), full["prim_id"])
        if fields & _capi.VRH_RT_OCC:
            assert np.array_equal(np.load(tmp_path / f"occ{f}.npy"), full["occ"])
        if fields & _capi.VRH_RT_T:
            assert np.array_equal(np.load(tmp_path / f"t{f}.npy").view(np.uint32), full["t"].view(np.uint32))
        assert np.array_equal(np.load(tmp_path / f"color{f}.npy").view(np.uint32), full["color"].view(np.uint32))
    assert st[0] == world                      # max over ranks
    assert int(st[1]) == rays                  # rays summed over ranks = every frame


def test_plan_known_values():
    """libvrh's plan against hand-derived values (8-row bands dealt round-robin):
    an off-by-one anywhere in vrh_plan.h changes one of these."""
    # H = 36: 5 bands (the last one 4 rows); S = 2: shard 0 owns bands 0, 2, 4, shard 1 bands 1, 3
    assert [multigpu.shard_bands(36, s, 2) for s in range(2)] == [3, 2]
    assert multigpu.rows_max(36, 2) == 24
    assert multigpu.packed_rows(36, 0, 2).tolist() == list(range(0, 8)) + list(range(16, 24)) + \
        list(range(32, 36)) + [-1] * 4
    assert multigpu.packed_rows(36, 1, 2).tolist() == list(range(8, 16)) + list(range(24, 32)) + [-1] * 8
    # S = 8 over 2 bands: shards 2..7 own nothing
    assert [multigpu.shard_bands(16, s, 8) for s in range(8)] == [1, 1, 0, 0, 0, 0, 0, 0]
    # N = 3 ranks, S = 5 shards: rank r sends r, r + 3; the root receives s from s % 3
    assert [multigpu.owned_shards(r, 3, 5) for r in range(3)] == [[0, 3], [1, 4], [2]]
    assert [multigpu.shard_owner(s, 3) for s in range(5)] == [0, 1, 2, 0, 1]
    # N = 3, S = 2: rank 2 owns nothing
    assert multigpu.owned_shards(2, 3, 2) == []
    # 4 x 36 image, 2 shards of 24 rows, 3 frames: [prim ids | masks | t] of 288 pixels
    w = multigpu.wire_layout(FIELDS_ALL, 4, 36, 3, 2)
    px = 3 * 24 * 4
    assert (w.rows, w.prim_id, w.occ, w.t, w.shard_bytes) == (24, 0, 4 * px, 5 * px, 9 * px)
    assert (w.color, w.code) == (_capi.VRH_WIRE_ABSENT, _capi.VRH_WIRE_ABSENT) and w.derive == 1
    w = multigpu.wire_layout(FIELDS_COLOR, 4, 36, 3, 2)
    assert (w.code, w.shard_bytes, w.prim_id) == (0, px, _capi.VRH_WIRE_ABSENT)


def test_unshard_of_synthetic_shards():
    """vrh_unshard_host on shards whose prim ids encode (frame, image row, x): every pixel lands on
    its own row; colour re-derived from the code byte."""
    Wd, Hd, S, F = 5, 37, 3, 2
    w = multigpu.wire_layout(FIELDS_IDS, Wd, Hd, F, S, bg=BG)
    g = np.zeros((S, w.shard_bytes), np.uint8)
    for s in range(S):
        rows = multigpu.packed_rows(Hd, s, S)
        pid = multigpu.field(g[s], w, "prim_id", F, Wd, np.uint32)
        occ = multigpu.field(g[s], w, "occ", F, Wd, np.uint8)
        for f in range(F):
            for lr, y in enumerate(rows):
                pid[f, lr * Wd:(lr + 1) * Wd] = 0xFFFFFFFF if y < 0 else (f * 1000 + y) * 8 + np.arange(Wd)
                occ[f, lr * Wd:(lr + 1) * Wd] = 0 if y < 0 else (y * 7 + f) & 0xFF
    for f in range(F):
        out = multigpu.unshard(g, w, FIELDS_IDS, Wd, Hd, S, f, bg=BG)
        y, x = np.divmod(np.arange(Wd * Hd), Wd)
        assert np.array_equal(out["prim_id"], ((f * 1000 + y) * 8 + x).astype(np.uint32))
        assert np.array_equal(out["occ"], ((y * 7 + f) & 0xFF).astype(np.uint8))
        k = np.array([bin(v).count("1") for v in out["occ"]])
        grey = np.float32(1.0)
        levels = [grey]
        for _ in range(8):
            grey = np.float32(grey - np.float32(1.0 / 8))
            levels.append(grey)
        assert np.array_equal(out["color"][:, 0], np.array(levels, np.float32)[k])


def test_wire_layout_fields():
    """What crosses the wire per target (vrh_plan.h layout_for): colour-only -> 1 code byte;
    colour + ids -> prim id + mask (colour re-derived); t adds 4 B; >8 AO samples carry no mask."""
    def per_px(fields, samples=8):
        w = multigpu.wire_layout(fields, W, H, 1, 3, samples=samples)
        return w.shard_bytes // (w.rows * W)
    assert per_px(FIELDS_COLOR) == 1
    assert per_px(FIELDS_IDS) == 5
    assert per_px(FIELDS_ALL) == 9
    assert per_px(_capi.VRH_RT_COLOR, samples=16) == 16      # colour itself: the code cannot hold it
    assert per_px(_capi.VRH_RT_OCC | _capi.VRH_RT_PRIM_ID, samples=16) == 4


def test_pack_code_counts_occluded_samples():
    pid = np.array([0xFFFFFFFF, 3, 4, 5], np.uint32)
    occ = np.array([0xFF, 0, 0b1011, 0xFF], np.uint8)
    assert multigpu.pack_code(pid, occ).tolist() == [0xFF, 0, 3, 8]
    assert multigpu.pack_code(pid).tolist() == [0xFF, 0, 0, 0]


def test_band_partition_covers_image_once():
    for Hh in (1, 17, 90, 1080):
        # vrh_shard_bands (the count the device uses) sums to the image's bands
        for shards in (1, 2, 3, 8, 135):
            assert sum(multigpu.shard_bands(Hh, s, shards) for s in range(shards)) == (Hh + 7) // 8
        for shards in (1, 2, 3, 4, 8, 135):
            seen = np.concatenate([multigpu.packed_rows(Hh, s, shards) for s in range(shards)])
            seen = seen[seen >= 0]
            assert np.array_equal(np.sort(seen), np.arange(Hh))
            assert all(len(multigpu.packed_rows(Hh, s, shards)) <= multigpu.rows_max(Hh, shards) for s in range(shards))


def test_exchange_plan_pairs_every_send_with_a_receive():
    for world in (1, 2, 3, 8):
        for shards in (1, max(world - 1, 1), world, world + 1, 3 * world):
            recvs = multigpu.exchange_plan(0, world, shards)[1]
            assert [s for s, _ in recvs] == list(range(shards))
            for rank in range(world):
                sends = multigpu.exchange_plan(rank, world, shards)[0]
                # per peer, the root's receives from `rank` list the same shards in the same order
                assert [s for s, _ in sends] == [s for s, p in recvs if p == rank]


def test_unshard_host_rejects_mismatched_wire_and_empty_width():
    """vrh_unshard_host checks that the wire layout is the one the fields and kernel give, and that the
    image has a width (a zero width or an empty wire layout was a division by zero)."""
    Wd, Hd, S, F = 5, 37, 3, 2
    w_ids = multigpu.wire_layout(FIELDS_IDS, Wd, Hd, F, S, bg=BG)
    g = np.zeros((S, w_ids.shard_bytes), np.uint8)
    # the same bytes read as a colour-only gather: another layout -> refused, not re-derived quietly
    with pytest.raises(_capi.VrhError):
        multigpu.unshard(g, w_ids, FIELDS_COLOR, Wd, Hd, S, 0, bg=BG)
    with pytest.raises(_capi.VrhError):
        multigpu.unshard(g, w_ids, FIELDS_IDS, 0, Hd, S, 0, bg=BG)
    multigpu.unshard(g, w_ids, FIELDS_IDS, Wd, Hd, S, F - 1, bg=BG)      # the matching call still works
