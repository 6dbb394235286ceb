"""CPU: the oracle's frame-number sampler offset, BVH-ref lists and scissor box against fixtures the
reference harness produced (tests/golden/make_golden.py --frames / --list).

* frame cases: the golden AO frame of frame number n (vrh.h vrh_render: the Appendix-A counter
  offset by n * 0x9E3779B1; frame 0 is the parity frame of test_oracle.py);
* list cases: closest_hit / any_hit over a list of two BVH refs (traverse_linear.inl:76-141) --
  the scene split by prim_id parity, each half built by the reference's own builder -- rendered by
  the reference's tiled_sched with a scissor box (tiled_sched.inl:244-260; pixels outside the box
  untouched).
"""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FRAME_CASES = ["frame7_hf64_160x90", "frame1_hf200_320x180"]
LIST_CASES = ["list_hf64_160x90", "list_hf200_320x180", "list_cornell12_128"]


def list_members(O, ref, scene_name):
    """The two BVHs of a list fixture as oracle Scenes (normals by prim_id on the first)."""
    kind, prims_all = O.gen_prims(scene_name)
    normals = O.face_normals(prims_all)
    members = []
    for k in (0, 1):
        prims = ref[f"bvh{k}_prims"].view(O.TRI_DTYPE)
        nodes = ref[f"bvh{k}_nodes"].view(O.NODE_DTYPE)
        idx = ref[f"bvh{k}_indices"]
        # the harness built each half with the reference builder: the oracle's builder agrees
        n2, i2, depth = O.build_bvh(prims, O.VO_TRI)
        assert np.array_equal(n2.view(np.uint32), nodes.view(np.uint32)) and np.array_equal(i2, idx)
        members.append(O.Scene(scene_name, O.VO_TRI, prims, nodes, idx, normals if k == 0 else None, depth))
    return members


@pytest.mark.parametrize("case", FRAME_CASES)
def test_frame_number_offsets_the_ao_sampler(oracle_mod, golden, case):
    O = oracle_mod
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    sc = O.make_scene(g["scene"])
    cam = O.scene_camera(g["scene"], g["W"], g["H"])
    out = O.render(sc, cam, mode=O.VO_MODE_AO, frame_num=g["frame"])
    assert np.array_equal(out["prim_id"], ref["prim_id"])
    assert np.array_equal(out["occ"], ref["occ"])
    assert np.array_equal(out["color"].view(np.uint32), ref["color"].view(np.uint32))
    # a different frame number is a different AO sample set (frame 0 = the parity fixture)
    base = np.load(os.path.join(HERE, "golden", g["scene"] + f"_{g['W']}x{g['H']}.npz"))
    assert not np.array_equal(out["occ"], base["occ"])
    assert np.array_equal(out["prim_id"], base["prim_id"])


def test_frame_number_full_size_sample(oracle_mod, golden):
    O = oracle_mod
    g = golden["frame3_hf1M"]
    ref = np.load(os.path.join(HERE, "golden", "frame3_hf1M.npz"))
    sc = O.make_scene("hf1M")
    cam = O.scene_camera("hf1M", 1920, 1080)
    out = O.render_pixels(sc, cam, ref["pixels"], mode=O.VO_MODE_AO, frame_num=3)
    assert np.array_equal(out["prim_id"], ref["prim_id"])
    assert np.array_equal(out["occ"], ref["occ"])
    assert np.array_equal(out["color"].view(np.uint32), ref["color"].view(np.uint32))


@pytest.mark.parametrize("case", LIST_CASES)
def test_bvh_list_with_scissor_matches_reference(oracle_mod, golden, case):
    O = oracle_mod
    g = golden[case]
    ref = np.load(os.path.join(HERE, "golden", case + ".npz"))
    members = list_members(O, ref, g["scene"])
    cam = O.scene_camera(g["scene"], g["W"], g["H"])
    out = O.render(members, cam, mode=O.VO_MODE_AO, frame_num=g["frame"], scissor=tuple(g["scissor"]))
    assert np.array_equal(out["prim_id"], ref["prim_id"]), f"{(out['prim_id'] != ref['prim_id']).sum()} prim ids differ"
    assert np.array_equal(out["t"].view(np.uint32), ref["t"].view(np.uint32))
    assert np.array_equal(out["list_index"], ref["leaf_pos"])
    assert np.array_equal(out["occ"], ref["occ"])
    assert np.array_equal(out["color"].view(np.uint32), ref["color"].view(np.uint32))
    # the scissor box really clips: nothing outside it was written
    W, H = g["W"], g["H"]
    x0, y0, x1, y1 = g["scissor"]
    inside = np.zeros((H, W), bool)
    inside[y0:y1, x0:x1] = True
    assert (ref["prim_id"].reshape(H, W)[~inside] == 0xFFFFFFFF).all()
    assert int((ref["prim_id"] != 0xFFFFFFFF).sum()) == g["hits"]
