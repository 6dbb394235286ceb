"""GPU: failure containment of the RCCL render groups (vrh.h vrh_group_join_timeout).

The first multi-GPU run must end with an error when a rank is missing, not hang until the driver's
time limit: the communicator is non-blocking, every wait on a peer is polled against the group's
deadline, and a missed deadline aborts the communicator (ncclCommAbort) and reports VRH_ERR_TIMEOUT.
On a one-GPU box the missing peer is simulated by a two-rank group whose second rank never joins.
"""
import time

import numpy as np
import pytest

import visionaray_amd as va
from visionaray_amd import _capi, scenes

pytestmark = pytest.mark.gpu


def test_join_with_a_missing_peer_fails_within_the_deadline(ctx):
    uid = va.render_group.unique_id()
    t0 = time.monotonic()
    with pytest.raises(_capi.VrhError) as e:
        va.render_group(ctx, 2, 0, uid, timeout_ms=3000)
    dt = time.monotonic() - t0
    assert e.value.code == _capi.VRH_ERR_TIMEOUT, str(e.value)
    assert 2.5 < dt < 30.0, f"join gave up after {dt:.1f} s"
    assert "aborted" in str(e.value)


def test_context_and_groups_work_after_a_failed_join(ctx):
    """The abort leaves the device usable: a frame renders, and a fresh (one-rank) group gathers."""
    uid = va.render_group.unique_id()
    with pytest.raises(_capi.VrhError):
        va.render_group(ctx, 2, 1, uid, timeout_ms=1500)
    name, W, H = "hf64", 160, 90
    prims = scenes.primitives(name)
    dev = va.hip_index_bvh(ctx, va.build_index_bvh(prims), scenes.normals_for(prims))
    cam, _, _ = scenes.scene_camera(name, W, H)
    basis = cam.basis(W, H)
    k = va.ao_kernel(dev)
    ref = va.hip_buffer_rt(ctx, W, H)
    va.render(ctx, dev, ref, basis, k)
    want = ref.download()
    g = va.render_group(ctx, 1, 0, va.render_group.unique_id(), timeout_ms=5000)
    assert not g.failed
    dst = va.hip_buffer_rt(ctx, W, H)
    g.render(dev, k, dst, [basis], shards=3)
    g.sync()
    got = dst.download()
    g.close()
    for key in ("prim_id", "occ"):
        assert np.array_equal(got[key], want[key])
    assert np.array_equal(got["color"].view(np.uint32), want["color"].view(np.uint32))


def test_group_timeout_argument_checked(ctx):
    g = va.render_group(ctx, 1, 0, va.render_group.unique_id())
    try:
        with pytest.raises(_capi.VrhError):
            g.set_timeout(0)
        g.set_timeout(250)
        assert not g.failed
    finally:
        g.close()
