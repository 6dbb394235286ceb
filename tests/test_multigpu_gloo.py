"""CPU, world_size 2 and 3 over gloo: the protocol of libvrh's render groups (vrh_render_sharded,
restated in visionaray_amd/multigpu.py) -- shard ownership s -> rank s % N, packed shard buffers
of several frames on the wire as [prim ids | AO masks] (or one colour code byte per pixel), point-to-point sends / receives paired in
plan order, the root's un-interleave and colour re-derivation, the ray-count sum and max-over-ranks
timing of bench.py -- reproduces the single-process frames bit for bit, including S > N shards.
The per-rank renderer is the oracle restricted to the shard's rows; on the GPU box the same
protocol runs inside libvrh over RCCL (tests/test_gpu_group.py: a one-rank group with S shards)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from visionaray_amd import multigpu

SCENE, W, H, FRAMES, FRAME0 = "hf64", 160, 90, 2, 4
BG = (0.1, 0.2, 0.3, 1.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, shards, port, outdir, ids=True):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        sc = O.make_scene(SCENE)
        cam = O.scene_camera(SCENE, W, H)
        rm = multigpu.rows_max(H, shards)
        lay, nbytes = multigpu.wire_layout(FRAMES, rm, W, ids=ids)
        sends, recvs = multigpu.exchange_plan(rank, world, shards)
        rays = 0
        bufs = []
        for s, _ in sends:                           # render every owned shard, packed
            buf = np.zeros(nbytes, np.uint8)
            if ids:
                pid = buf[lay["pid"][0]:lay["pid"][0] + lay["pid"][1]].view(np.uint32).reshape(FRAMES, rm * W)
                occ = buf[lay["occ"][0]:lay["occ"][0] + lay["occ"][1]].reshape(FRAMES, rm * W)
            else:   # rendered into a work buffer, then packed to the code byte
                pid = np.empty((FRAMES, rm * W), np.uint32)
                occ = np.zeros((FRAMES, rm * W), np.uint8)
            pid[:] = 0xFFFFFFFF
            for f in range(FRAMES):
                for lr, y in enumerate(multigpu.packed_rows(H, s, shards)):
                    if y < 0:
                        continue
                    out = O.render(sc, cam, mode=O.VO_MODE_AO, rows=(int(y), int(y) + 1), threads=1,
                                   frame_num=FRAME0 + f)
                    pid[f, lr * W:(lr + 1) * W] = out["prim_id"][y * W:(y + 1) * W]
                    occ[f, lr * W:(lr + 1) * W] = out["occ"][y * W:(y + 1) * W]
                    rays += out["rays"]
            if not ids:
                buf[:] = multigpu.pack_code(pid.reshape(-1), occ.reshape(-1))
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
                    t = torch.empty(nbytes, dtype=torch.uint8)
                    dist.recv(t, src=peer)
                    gathered[s] = t.numpy()
        for r in reqs:
            r.wait()
        stats = torch.tensor([float(rank + 1), float(rays)], dtype=torch.float64)
        mx, sm = stats.clone(), stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        if rank == 0:
            for f in range(FRAMES):
                if not ids:
                    gc = gathered.reshape(shards, FRAMES, rm * W)[:, f]
                    code = multigpu.unshard_host(gc, W, H, shards)
                    np.save(os.path.join(outdir, f"color{f}.npy"), multigpu.derive_colour_code(code, BG))
                    continue
                gp = gathered[:, lay["pid"][0]:lay["pid"][0] + lay["pid"][1]].view(np.uint32).reshape(shards, FRAMES, rm * W)[:, f]
                go = gathered[:, lay["occ"][0]:lay["occ"][0] + lay["occ"][1]].reshape(shards, FRAMES, rm * W)[:, f]
                pid = multigpu.unshard_host(gp, W, H, shards)
                occ = multigpu.unshard_host(go, W, H, shards)
                np.save(os.path.join(outdir, f"pid{f}.npy"), pid)
                np.save(os.path.join(outdir, f"occ{f}.npy"), occ)
                np.save(os.path.join(outdir, f"color{f}.npy"), multigpu.derive_colour(pid, occ, BG))
            np.save(os.path.join(outdir, "stats.npy"), np.array([mx[0].item(), sm[1].item()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shards,ids", [(2, 2, True), (3, 3, True), (2, 5, True), (2, 3, False)])
def test_sharded_exchange_equals_single_frames(tmp_path, oracle_mod, world, shards, ids):
    """ids=False: a colour-only target, one code byte per pixel on the wire (bench.py's N > 1 default)."""
    O = oracle_mod
    mp.start_processes(_worker, args=(world, shards, _free_port(), str(tmp_path), ids), nprocs=world, join=True,
                       start_method="spawn")
    st = np.load(tmp_path / "stats.npy")
    rays = 0
    for f in range(FRAMES):
        full = O.render(O.make_scene(SCENE), O.scene_camera(SCENE, W, H), mode=O.VO_MODE_AO, frame_num=FRAME0 + f)
        rays += full["rays"]
        if ids:
            assert np.array_equal(np.load(tmp_path / f"pid{f}.npy"), full["prim_id"])
            assert np.array_equal(np.load(tmp_path / f"occ{f}.npy"), full["occ"])
        assert np.array_equal(np.load(tmp_path / f"color{f}.npy").view(np.uint32), full["color"].view(np.uint32))
    assert st[0] == world                      # max over ranks
    assert int(st[1]) == rays                  # rays summed over ranks = every frame


def test_band_partition_covers_image_once():
    for Hh in (1, 17, 90, 1080):
        for shards in (1, 2, 3, 4, 8, 135):
            seen = np.concatenate([multigpu.packed_rows(Hh, s, shards) for s in range(shards)])
            seen = seen[seen >= 0]
            assert np.array_equal(np.sort(seen), np.arange(Hh))
            assert all(len(multigpu.packed_rows(Hh, s, shards)) <= multigpu.rows_max(Hh, shards) for s in range(shards))


def test_exchange_plan_pairs_every_send_with_a_receive():
    for world in (1, 2, 3, 8):
        for shards in (1, world, world + 1, 3 * world):
            recvs = multigpu.exchange_plan(0, world, shards)[1]
            assert [s for s, _ in recvs] == list(range(shards))
            for rank in range(world):
                sends = multigpu.exchange_plan(rank, world, shards)[0]
                # per peer, the root's receives from `rank` list the same shards in the same order
                assert [s for s, _ in sends] == [s for s, p in recvs if p == rank]
