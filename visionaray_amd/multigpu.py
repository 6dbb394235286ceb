"""Image-tile sharding across GPUs: the render-group plan libvrh runs
(vrh.h vrh_render_sharded, visionaray_amd/csrc/vrh_group.hip), exposed from the library itself.

Every function here is a thin ctypes call into libvrh's host exports (vrh_group_shards_of,
vrh_group_shard_owner, vrh_group_wire_layout, vrh_shard_packed_rows, vrh_pack_codes_host,
vrh_unshard_host), which run the same code (csrc/vrh_plan.h) as the GPU path -- so the
multi-process CPU tests (tests/test_multigpu_gloo.py) drive the protocol the GPUs run, not a
restatement of it:

* 8-row bands are dealt round-robin to S shards (band b -> shard b % S); shard s is rendered by rank
  s % N, packed: its bands back to back in a buffer of `rows` rows (shard 0 owns the most bands).
* On the wire one shard is [prim ids | AO masks | t | colour | codes] of every frame (wire_layout);
  a colour-only target of a built-in kernel sends one code byte per pixel (0xFF miss, else the
  number of occluded AO samples). Rank r sends its shards r, r + N, ... in that order; the root
  receives shard s from rank s % N for s = 0, 1, ..., so sends and receives pair up in order per peer.
* The root un-interleaves every frame and re-derives the built-in colour (unshard).

No device is needed for any of these calls.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi

BAND = _capi.VRH_BAND_ROWS


def _kernel_desc(ao=True, samples=8, bg=(0.0, 0.0, 0.0, 1.0)):
    k = _capi.vrh_kernel_desc()
    k.kind = _capi.VRH_KERNEL_AO if ao else _capi.VRH_KERNEL_PRIMARY
    k.samples = samples
    for i in range(4):
        k.bg[i] = bg[i]
    return k


def shard_bands(height, shard, shards):
    """Number of bands shard owns (vrh_shard_bands)."""
    return int(_capi.lib().vrh_shard_bands(height, shard, shards))


def rows_max(height, shards):
    """Rows of every packed shard buffer (shard 0 owns the most bands)."""
    return BAND * shard_bands(height, 0, shards)


def packed_rows(height, shard, shards):
    """Image rows of a packed shard, in packed order (-1 for padding rows past the image)."""
    out = np.empty(rows_max(height, shards), np.int32)
    _capi.check("vrh_shard_packed_rows", height, shard, shards, out.ctypes.data_as(C.POINTER(C.c_int32)))
    return out.astype(np.int64)


def owned_shards(rank, nranks, shards):
    """Shards rank renders, in the order it sends them (vrh_group_shards_of)."""
    buf = (C.c_uint32 * max(shards, 1))()
    n = _capi.lib().vrh_group_shards_of(nranks, rank, shards, buf, max(shards, 1))
    return [int(buf[j]) for j in range(n)]


def shard_owner(shard, nranks):
    return int(_capi.lib().vrh_group_shard_owner(nranks, shard))


def exchange_plan(rank, nranks, shards):
    """(sends, receives) of one rank in one vrh_render_sharded call: sends = [(shard, peer 0)] in
    send order; receives (root only) = [(shard, peer)] in receive order."""
    sends = [(s, 0) for s in owned_shards(rank, nranks, shards)]
    recvs = [(s, shard_owner(s, nranks)) for s in range(shards)] if rank == 0 else []
    return sends, recvs


def wire_layout(fields, width, height, frames, shards, ao=True, samples=8, bg=(0.0, 0.0, 0.0, 1.0)):
    """The packed-shard layout of a root target with buffers `fields` (VRH_RT_* bits) for the
    built-in AO (or primary-visibility) kernel: a _capi.vrh_wire_layout (byte offsets, absent fields
    VRH_WIRE_ABSENT; shard_bytes; rows per shard and frame; derive)."""
    w = _capi.vrh_wire_layout()
    k = _kernel_desc(ao, samples, bg)
    _capi.check("vrh_group_wire_layout", fields, C.byref(k), width, height, frames, shards, C.byref(w))
    return w


def field(buf, wire, name, frames, width, dtype):
    """View of field `name` ("prim_id", "occ", "t", "code") of a packed shard as (frames, rows*width)."""
    off = getattr(wire, name)
    assert off != _capi.VRH_WIRE_ABSENT, f"{name} is not on the wire"
    n = frames * wire.rows * width * np.dtype(dtype).itemsize
    return buf[off:off + n].view(dtype).reshape(frames, wire.rows * width)


def pack_code(pid, occ=None):
    """One byte per rendered pixel (vrh_pack_codes_host): 0xFF on a miss, else the number of
    occluded AO samples (0 without an AO mask)."""
    pid = np.ascontiguousarray(pid, np.uint32)
    code = np.empty(len(pid), np.uint8)
    o = None if occ is None else np.ascontiguousarray(occ, np.uint8)
    _capi.check("vrh_pack_codes_host", pid.ctypes.data, None if o is None else o.ctypes.data, code.ctypes.data,
                len(pid))
    return code


def unshard(gathered, wire, fields, width, height, shards, frame, ao=True, samples=8, bg=(0.0, 0.0, 0.0, 1.0)):
    """The root's un-interleave of one frame from the S gathered shards (a (S, shard_bytes) uint8
    array) into full-image buffers (vrh_unshard_host): {"color", "prim_id", "occ", "t"} for the
    fields the root target holds."""
    g = np.ascontiguousarray(gathered, np.uint8)
    assert g.shape == (shards, wire.shard_bytes), (g.shape, shards, wire.shard_bytes)
    n = width * height
    out = {}
    if fields & _capi.VRH_RT_COLOR:
        out["color"] = np.zeros((n, 4), np.float32)
    if fields & _capi.VRH_RT_PRIM_ID:
        out["prim_id"] = np.zeros(n, np.uint32)
    if fields & _capi.VRH_RT_OCC:
        out["occ"] = np.zeros(n, np.uint8)
    if fields & _capi.VRH_RT_T:
        out["t"] = np.zeros(n, np.float32)
    k = _kernel_desc(ao, samples, bg)
    ptr = lambda key: out[key].ctypes.data if key in out else None   # noqa: E731
    _capi.check("vrh_unshard_host", g.ctypes.data, C.byref(wire), width, height, shards, frame, fields, C.byref(k),
                ptr("color"), ptr("prim_id"), ptr("occ"), ptr("t"))
    return out
