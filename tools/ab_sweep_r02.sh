#!/bin/bash
# round-2 re-sweeps of launch defaults (tools/ab_builds.sh launch variants); logs under gpurun_out/
#   ab19: primary (sph1M, hf1M) and AO (hf1M) knobs; ab20: the primary refill threshold, 20 and 1
#   frames per launch; ab21: the new default against the old one; ab28: tile order with frames in flight
case "${1:-ab21}" in
ab19)
  export VRH_AB='[{"name":"default"},{"name":"occ5","waves_per_simd":5},{"name":"occ8","waves_per_simd":8},{"name":"dcap4","descent_cap":4},{"name":"dcap16","descent_cap":16},{"name":"refill4","refill_min":4},{"name":"refill16","refill_min":16},{"name":"nopop","pop_on_miss":2},{"name":"scalar off","scalar_fetch":2},{"name":"global queue","xcd_queues":2}]'
  SCENES="sph1M hf1M" KERNEL=primary REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab19_primary.log 2>&1 || exit $?
  export VRH_AB='[{"name":"default"},{"name":"refill16","refill_min":16},{"name":"refill24","refill_min":24},{"name":"refill40","refill_min":40},{"name":"refill48","refill_min":48},{"name":"occ6","waves_per_simd":6},{"name":"global queue","xcd_queues":2},{"name":"dcap8","descent_cap":8}]'
  SCENES="hf1M" KERNEL=ao REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab19_ao.log 2>&1 ;;
ab20)
  export VRH_AB='[{"name":"default"},{"name":"refill8","refill_min":8},{"name":"refill12","refill_min":12},{"name":"refill16","refill_min":16},{"name":"refill24","refill_min":24},{"name":"refill32","refill_min":32}]'
  SCENES="sph1M hf1M hf10M" KERNEL=primary REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab20_refill.log 2>&1 || exit $?
  SCENES="sph1M hf1M" KERNEL=primary BATCH=1 REPS=1 ROUNDS=4 bash tools/ab_builds.sh > gpurun_out/ab20_refill_f1.log 2>&1 ;;
ab21)
  export VRH_AB='[{"name":"warm-up"},{"name":"default (16)"},{"name":"refill1 (old)","refill_min":1},{"name":"default again"}]'
  SCENES="sph1M hf1M hf10M" KERNEL=primary REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab21_refill_default.log 2>&1 ;;
ab22)
  export VRH_AB='[{"name":"warm-up"},{"name":"default"},{"name":"refill24","refill_min":24},{"name":"refill40","refill_min":40},{"name":"dcap16","descent_cap":16},{"name":"occ6","waves_per_simd":6},{"name":"stack12","stack_cap":12},{"name":"stack16","stack_cap":16},{"name":"stack24","stack_cap":24},{"name":"nopop","pop_on_miss":2}]'
  SCENES="hf10M" KERNEL=ao REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab22_c4_defaults.log 2>&1 ;;
ab23)
  export VRH_AB='[{"name":"warm-up"},{"name":"default"},{"name":"refill16","refill_min":16},{"name":"refill24","refill_min":24},{"name":"refill48","refill_min":48},{"name":"occ6","waves_per_simd":6},{"name":"ungated","ao_gate":2},{"name":"binary","wide_anyhit":2},{"name":"global queue","xcd_queues":2},{"name":"default again"}]'
  SCENES="hf1M hf10M" KERNEL=ao BATCH=1 REPS=1 ROUNDS=5 bash tools/ab_builds.sh > gpurun_out/ab23_ao_single_frame.log 2>&1 ;;
ab28)
  # tile order with frames in flight: per-XCD strips (round-2 default) vs band-interleaved (band, frame) units
  export VRH_AB='[{"name":"warm-up"},{"name":"band-interleaved (auto)"},{"name":"strips","xcd_queues":1},{"name":"band-interleaved","xcd_queues":3},{"name":"strips again","xcd_queues":1}]'
  SCENES="hf1M hf10M" KERNEL=ao REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab28_tile_order_ao.log 2>&1 || exit $?
  SCENES="sph1M hf1M hf10M" KERNEL=primary REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab28_tile_order_primary.log 2>&1 ;;
ab29)
  # band-interleaved (queue = unit % 8) vs band-major per XCD (all frames of band b on queue b % 8;
  # the round-2 experiment build, option 4, removed after this A/B)
  export VRH_AB='[{"name":"warm-up"},{"name":"band-interleaved (auto)"},{"name":"band-major","xcd_queues":4},{"name":"strips","xcd_queues":1},{"name":"band-interleaved again","xcd_queues":3},{"name":"band-major again","xcd_queues":4}]'
  SCENES="hf1M hf10M" KERNEL=ao REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab29_band_major_ao.log 2>&1 || exit $?
  SCENES="sph1M hf1M hf10M" KERNEL=primary REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab29_band_major_primary.log 2>&1 ;;
ab30)
  # one frame per launch: strips (default) vs band-interleaved
  export VRH_AB='[{"name":"warm-up"},{"name":"strips (auto)"},{"name":"band-interleaved","xcd_queues":3},{"name":"strips again","xcd_queues":1},{"name":"band-interleaved again","xcd_queues":3}]'
  SCENES="hf1M hf10M" KERNEL=ao BATCH=1 REPS=1 ROUNDS=5 bash tools/ab_builds.sh > gpurun_out/ab30_tile_order_f1_ao.log 2>&1 || exit $?
  SCENES="sph1M hf1M" KERNEL=primary BATCH=1 REPS=1 ROUNDS=5 bash tools/ab_builds.sh > gpurun_out/ab30_tile_order_f1_primary.log 2>&1 ;;
ab31)
  # tile order with frames in flight and a moving camera (0.5 deg of orbit per frame): no two frames
  # of a launch share primary rays, so band-interleaving gets no credit from coinciding frames
  export VRH_AB='[{"name":"warm-up"},{"name":"band-interleaved (auto)"},{"name":"strips","xcd_queues":1},{"name":"band-interleaved again","xcd_queues":3},{"name":"strips again","xcd_queues":1}]'
  export VRH_AB_ORBIT=0.5
  SCENES="hf1M hf10M" KERNEL=ao REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab31_tile_order_orbit_ao.log 2>&1 || exit $?
  SCENES="hf1M hf10M" KERNEL=primary REPS=1 ROUNDS=3 bash tools/ab_builds.sh > gpurun_out/ab31_tile_order_orbit_primary.log 2>&1 ;;
esac
