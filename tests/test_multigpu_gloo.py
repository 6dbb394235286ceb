"""CPU, world_size 2 and 3 over gloo: the N>1 path of bench.py (band sharding, packed shard buffers,
gather to rank 0, un-interleave, ray-count sum and max-over-ranks timing) reproduces the
single-process frame bit for bit.  The per-rank renderer here is the oracle restricted to the
rank's rows (the GPU box runs the same plumbing with libvrh shards over RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from visionaray_amd import multigpu

SCENE, W, H = "hf64", 160, 90


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        sc = O.make_scene(SCENE)
        cam = O.scene_camera(SCENE, W, H)
        rm = multigpu.rows_max(H, world)
        rows = multigpu.packed_rows(H, rank, world)
        loc_color = np.zeros((rm * W, 4), np.float32)
        loc_pid = np.full(rm * W, 0xFFFFFFFF, np.uint32)
        rays = 0
        for lr, y in enumerate(rows):
            if y < 0:
                continue
            out = O.render(sc, cam, mode=O.VO_MODE_AO, rows=(int(y), int(y) + 1), threads=1)
            loc_color[lr * W:(lr + 1) * W] = out["color"][y * W:(y + 1) * W]
            loc_pid[lr * W:(lr + 1) * W] = out["prim_id"][y * W:(y + 1) * W]
            rays += out["rays"]
        tc = torch.from_numpy(loc_color)
        tp = torch.from_numpy(loc_pid.view(np.int32))
        outs = None
        if rank == 0:
            outs = [torch.empty((world,) + tuple(tc.shape), dtype=tc.dtype),
                    torch.empty((world,) + tuple(tp.shape), dtype=tp.dtype)]
        multigpu.gather_to_root(dist, [tc, tp], rank, world, outs)
        stats = torch.tensor([float(rank + 1), float(rays)], dtype=torch.float64)
        mx, sm = stats.clone(), stats.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        if rank == 0:
            color = multigpu.unshard_host(outs[0].numpy(), W, H, world)
            pid = multigpu.unshard_host(outs[1].numpy().view(np.uint32), W, H, world)
            np.save(os.path.join(outdir, "color.npy"), color)
            np.save(os.path.join(outdir, "pid.npy"), pid)
            np.save(os.path.join(outdir, "stats.npy"), np.array([mx[0].item(), sm[1].item()]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_gather_equals_single_frame(tmp_path, oracle_mod, world):
    O = oracle_mod
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    full = O.render(O.make_scene(SCENE), O.scene_camera(SCENE, W, H), mode=O.VO_MODE_AO)
    color = np.load(tmp_path / "color.npy")
    pid = np.load(tmp_path / "pid.npy")
    st = np.load(tmp_path / "stats.npy")
    assert np.array_equal(pid, full["prim_id"])
    assert np.array_equal(color.view(np.uint32), full["color"].view(np.uint32))
    assert st[0] == world                      # max over ranks
    assert int(st[1]) == full["rays"]          # rays summed over ranks = whole frame


def test_band_partition_covers_image_once():
    for Hh in (1, 17, 90, 1080):
        for world in (1, 2, 3, 4, 8):
            seen = np.concatenate([multigpu.packed_rows(Hh, r, world) for r in range(world)])
            seen = seen[seen >= 0]
            assert np.array_equal(np.sort(seen), np.arange(Hh))
            assert all(len(multigpu.packed_rows(Hh, r, world)) <= multigpu.rows_max(Hh, world) for r in range(world))
