mkdir -p gpurun_out
export VRH_AB='[{"name":"row-major"},{"name":"column-major","tile_order":2},{"name":"col+global queue","tile_order":2,"xcd_queues":2}]'
timeout -k 10 300 python tools/ab_variants.py hf1M 4 > gpurun_out/ab1_hf1M.log 2>&1 || exit $?
VRH_AB_BATCH=8 timeout -k 10 300 python tools/ab_variants.py hf10M 3 > gpurun_out/ab1_hf10M.log 2>&1 || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py hf1M 4 > gpurun_out/ab1_hf1M_primary.log 2>&1 || exit $?
VRH_AB_KERNEL=primary timeout -k 10 300 python tools/ab_variants.py sph1M 4 > gpurun_out/ab1_sph1M.log 2>&1 || exit $?
tail -5 gpurun_out/ab1_*.log
