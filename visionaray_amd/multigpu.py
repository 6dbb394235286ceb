"""Image-tile sharding across GPUs: one process per GPU, 8-row bands dealt
round-robin (band b -> rank b % N; interleaved so horizon and terrain rows balance), packed shard
framebuffers gathered to rank 0 over RCCL (torch.distributed "nccl"; "gloo" in the CPU tests) and
un-interleaved there.

The device un-interleave is vrh_unshard (HIP); unshard_host() is its host statement, used by the
multi-process CPU tests and as the specification of the mapping.
"""
from __future__ import annotations

import numpy as np

BAND = 8    # VRH_BAND_ROWS: one row of 8x8 wave tiles (1080 rows over 8 GPUs balance within 1 %)


def bands(height):
    return (height + BAND - 1) // BAND


def shard_bands(height, rank, world):
    """Number of bands rank owns (same as vrh_shard_bands)."""
    nb = bands(height)
    if rank >= world or rank >= nb:
        return 0
    return (nb - rank + world - 1) // world


def rows_max(height, world):
    """Rows of the packed shard buffer every rank allocates (rank 0 owns the most bands)."""
    return BAND * shard_bands(height, 0, world)


def packed_rows(height, rank, world):
    """Image rows of rank's packed shard, in packed order (-1 for padding rows past the image)."""
    out = []
    for lb in range(shard_bands(height, rank, world)):
        b = lb * world + rank
        for r in range(BAND):
            y = b * BAND + r
            out.append(y if y < height else -1)
    return np.array(out, dtype=np.int64)


def unshard_host(gathered, width, height, world):
    """gathered: (world, rows_max*width, ...) -> (height*width, ...), the vrh_unshard mapping."""
    rm = rows_max(height, world)
    g = np.asarray(gathered).reshape((world, rm, width) + tuple(np.asarray(gathered).shape[2:]))
    out = np.empty((height, width) + g.shape[3:], dtype=g.dtype)
    for rank in range(world):
        rows = packed_rows(height, rank, world)
        valid = rows >= 0
        out[rows[valid]] = g[rank, : len(rows)][valid]
    return out.reshape((height * width,) + g.shape[3:])


def gather_to_root(dist, tensors, rank, world, outs=None):
    """dist.gather each local tensor to rank 0 (outs: per tensor a (world, ...) tensor on rank 0).
    On RCCL this is a root-bound set of point-to-point transfers, one per xGMI link."""
    for i, t in enumerate(tensors):
        if rank == 0:
            dist.gather(t, gather_list=list(outs[i].unbind(0)), dst=0)
        else:
            dist.gather(t, dst=0)
