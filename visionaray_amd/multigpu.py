"""Image-tile sharding across GPUs: the host statement of the protocol libvrh's
render groups run (vrh.h vrh_render_sharded, visionaray_amd/csrc/vrh_group.hip).

* 8-row bands are dealt round-robin to S shards (band b -> shard b % S; interleaved so horizon and
  terrain rows balance); shard s is rendered by rank s % N, packed: its bands back to back in a
  buffer of rows_max(H, S) rows (shard 0 owns the most bands).
* On the wire one shard is [prim ids (u32) of every frame | AO masks (u8) of every frame | ...]
  (wire_layout), or for a colour-only target one code byte per pixel (0xFF miss, else the number
  of occluded AO samples, pack_code): the built-in colour depends on nothing else; rank r sends its shards r, r + N, ... in that order, the root receives shard s from
  rank s % N for s = 0, 1, ..., so sends and receives pair up in order per peer (exchange_plan).
* The root un-interleaves every frame (unshard_host = vrh_unshard's mapping) and re-derives the
  colour of the built-in kernels from prim id + AO mask (derive_colour) or from the code
  (derive_colour_code).

libvrh runs this with ncclSend / ncclRecv on the GPU; the multi-process CPU tests run it with gloo
point-to-point on oracle-rendered shards (tests/test_multigpu_gloo.py).
"""
from __future__ import annotations

import numpy as np

BAND = 8    # VRH_BAND_ROWS: one row of 8x8 wave tiles (1080 rows over 8 GPUs balance within 1 %)


def bands(height):
    return (height + BAND - 1) // BAND


def shard_bands(height, shard, shards):
    """Number of bands shard owns (same as vrh_shard_bands)."""
    nb = bands(height)
    if shard >= shards or shard >= nb:
        return 0
    return (nb - shard + shards - 1) // shards


def rows_max(height, shards):
    """Rows of every packed shard buffer (shard 0 owns the most bands)."""
    return BAND * shard_bands(height, 0, shards)


def packed_rows(height, shard, shards):
    """Image rows of a packed shard, in packed order (-1 for padding rows past the image)."""
    out = []
    for lb in range(shard_bands(height, shard, shards)):
        b = lb * shards + shard
        for r in range(BAND):
            y = b * BAND + r
            out.append(y if y < height else -1)
    return np.array(out, dtype=np.int64)


def owned_shards(rank, nranks, shards):
    """Shards rank renders, in the order it sends them: rank, rank + N, ..."""
    return list(range(rank, shards, nranks))


def exchange_plan(rank, nranks, shards):
    """(sends, receives) of one rank in one vrh_render_sharded call: sends = [(shard, peer 0)] in
    send order; receives (root only) = [(shard, peer)] in receive order."""
    sends = [(s, 0) for s in owned_shards(rank, nranks, shards)]
    recvs = [(s, s % nranks) for s in range(shards)] if rank == 0 else []
    return sends, recvs


def wire_layout(frames, rows, width, ao=True, ids=True):
    """Byte offsets of the fields of one packed shard of `frames` frames (built-in kernels with a
    colour + prim id (+ AO mask) target): {'pid': (offset, bytes), 'occ': ...}, total bytes.
    ids=False (a colour-only target, vrh_group.hip wire_layout::code): {'code': (0, px)}."""
    px = frames * rows * width
    if not ids:
        return {"code": (0, px)}, px
    lay = {"pid": (0, 4 * px)}
    if ao:
        lay["occ"] = (4 * px, px)
    return lay, sum(n for _, n in lay.values())


def unshard_host(gathered, width, height, shards):
    """gathered: (shards, rows_max*width, ...) -> (height*width, ...), the vrh_unshard mapping."""
    rm = rows_max(height, shards)
    g = np.asarray(gathered).reshape((shards, rm, width) + tuple(np.asarray(gathered).shape[2:]))
    out = np.empty((height, width) + g.shape[3:], dtype=g.dtype)
    for s in range(shards):
        rows = packed_rows(height, s, shards)
        valid = rows >= 0
        out[rows[valid]] = g[s, : len(rows)][valid]
    return out.reshape((height * width,) + g.shape[3:])


def derive_colour(pid, occ, bg, samples=8, ao=True):
    """The root's colour re-derivation (unshard_kernel): bg on a miss; 1 - k/samples for k occluded
    samples in sample order (ao/main.cpp:234-238), alpha 1; 1 for a primary-visibility hit."""
    pid = np.asarray(pid)
    out = np.empty((len(pid), 4), np.float32)
    out[:] = np.asarray(bg, np.float32)
    hit = pid != 0xFFFFFFFF
    clr = np.ones(len(pid), np.float32)
    if ao:
        step = np.float32(1.0) / np.float32(samples)
        for s in range(samples):
            occl = ((np.asarray(occ).astype(np.uint32) >> s) & 1).astype(bool)
            clr = np.where(occl, (clr - step).astype(np.float32), clr)
    out[hit, 0] = out[hit, 1] = out[hit, 2] = clr[hit]
    out[hit, 3] = 1.0
    return out


def pack_code(pid, occ=None):
    """One byte per rendered pixel (pack_code_kernel): 0xFF on a miss, else the number of occluded
    AO samples (0 without an AO mask)."""
    pid = np.asarray(pid)
    if occ is None:
        code = np.zeros(len(pid), np.uint8)
    else:
        code = np.unpackbits(np.asarray(occ, np.uint8)[:, None], axis=1).sum(axis=1).astype(np.uint8)
    code[pid == 0xFFFFFFFF] = 0xFF
    return code


def derive_colour_code(code, bg, samples=8, ao=True):
    """derive_colour from the code byte: bg on 0xFF; 1 - k/samples (k subtractions) for k occluded
    samples -- the same float sequence as subtracting in sample order."""
    code = np.asarray(code)
    out = np.empty((len(code), 4), np.float32)
    out[:] = np.asarray(bg, np.float32)
    hit = code != 0xFF
    clr = np.ones(len(code), np.float32)
    if ao:
        step = np.float32(1.0) / np.float32(samples)
        for s in range(samples):
            clr = np.where(code.astype(np.uint32) > s, (clr - step).astype(np.float32), clr)
    out[hit, 0] = out[hit, 1] = out[hit, 2] = clr[hit]
    out[hit, 3] = 1.0
    return out
