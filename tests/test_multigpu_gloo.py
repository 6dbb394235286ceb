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
