"""GPU: every traversal schedule and record width reaches the same bit-exact result.

The kernel has several ways to organise a wave's work (descent caps, pop on miss, refill thresholds,
the AO gate, VRH_OPT_WIDE_ANYHIT: 4-wide any-hit records, the stack's LDS share).  Only
the defaults run in test_gpu_parity.py; here the parity cases are re-run under each non-default
choice, on the same context, so none of the paths can drift from the reference.
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_gpu_parity as base  # noqa: E402
import visionaray_amd as va  # noqa: E402

pytestmark = pytest.mark.gpu

VARIANTS = {
    "step": {"ao_schedule": 3},
    "refill1": {"refill_min": 1},
    "global_queue": {"xcd_queues": 2},
    "band_interleaved_queues": {"xcd_queues": 3},
    "cluster_queues": {"xcd_queues": 4, "cluster_tiles": 5},
    "step_wide": {"ao_schedule": 3, "wide_anyhit": 1},
    "step_wide_exact": {"ao_schedule": 3, "wide_anyhit": 1, "exact_minmax": 1},
    "step_cap1": {"ao_schedule": 3, "descent_cap": 1},
    "step_refill24": {"ao_schedule": 3, "refill_min": 24},
    "step_cap3_wide": {"ao_schedule": 3, "descent_cap": 3, "wide_anyhit": 1},
    "step_pop_on_miss": {"ao_schedule": 3, "pop_on_miss": 1},
    "step_pop_cap2_wide": {"ao_schedule": 3, "pop_on_miss": 1, "descent_cap": 2, "wide_anyhit": 1},
    "scalar_off": {"ao_schedule": 3, "scalar_fetch": 2},
    "scalar_off_pop_cap2": {"ao_schedule": 3, "scalar_fetch": 2, "pop_on_miss": 1, "descent_cap": 2},
    "occ5": {"ao_schedule": 3, "waves_per_simd": 5},
    "occ6": {"ao_schedule": 3, "waves_per_simd": 6},
    # the primary-visibility defaults switched off (pop on miss, descent cap 8)
    "no_pop_uncapped": {"pop_on_miss": 2, "descent_cap": 1024, "refill_min": 16},
    "pop_cap10": {"pop_on_miss": 1, "descent_cap": 10},
    # the AO defaults switched off one by one (ao_gate + 4-wide any-hit + pop on miss)
    "ao_round1": {"ao_gate": 2, "wide_anyhit": 2, "pop_on_miss": 2},
    "ao_gate_binary": {"ao_gate": 1, "wide_anyhit": 2},
    "ao_ungated_wide": {"ao_gate": 2, "wide_anyhit": 1},
    "ao_cut_off": {"ao_cut": 2},
    "ao_cut_refill1_cap1": {"ao_cut": 1, "refill_min": 1, "descent_cap": 1},
    # the traversal stack mostly in the global overflow block (4 / 8 LDS entries per lane)
    "stack_lds4": {"stack_cap": 4},
    "stack_lds8_binary": {"stack_cap": 8, "wide_anyhit": 2},
    # scenes uploaded with the line-paired record layout (the option is read at upload)
    "pair_layout": {"pair_layout": 1},
}
OPTIONS = ("ao_schedule", "refill_min", "wide_anyhit", "exact_minmax", "descent_cap", "xcd_queues",
           "pop_on_miss", "scalar_fetch", "waves_per_simd", "pair_layout", "ao_gate",
           "stack_cap", "ao_cut", "cluster_tiles")


@pytest.fixture(params=sorted(VARIANTS))
def vctx(request, ctx):
    for k, v in VARIANTS[request.param].items():
        ctx.set_option(k, v)
    yield ctx
    for k in OPTIONS:
        ctx.set_option(k, 0)


@pytest.mark.parametrize("case", base.FULL_CASES)
def test_every_pixel(vctx, golden, case):
    base.test_every_pixel_matches_reference(vctx, golden, case)


@pytest.mark.parametrize("case", ["hf1M", "sph1M"])
def test_full_frame_hashes(vctx, golden, oracle_mod, case):
    base.test_full_frame_hashes_match_reference(vctx, golden, oracle_mod, case)


def test_random_soup(vctx, oracle_mod):
    base.test_random_soups_vs_oracle(vctx, oracle_mod, 1)


def test_edge_cases(vctx, oracle_mod):
    base.test_edge_cases_single_leaf_zero_dir_components_and_inside_sphere(vctx, oracle_mod)


def test_deep_comb(vctx, oracle_mod):
    base.test_deep_trees_overflow_stack_and_rejection(vctx, oracle_mod, 90)


def test_packed_shards(vctx):
    base.test_packed_shards_gather_to_identical_image(vctx, 3)


def test_removed_schedules_are_refused(ctx):
    """The item loop (round 2) and the cooperative fetch (round 1) were removed: asking for them is an
    error, not a silent fallback."""
    for opt, val in (("ao_schedule", 4), ("coop_fetch", 1)):
        with pytest.raises(va.VrhError):
            ctx.set_option(opt, val)
        ctx.set_option(opt, 0)
