set -o pipefail
export VRH_AB='[{"name":"default"},{"name":"waves6","waves_per_simd":6},{"name":"waves6 cap20","waves_per_simd":6,"stack_cap":20},{"name":"waves6 cap12","waves_per_simd":6,"stack_cap":12}]'
OUT=gpurun_out/s4 bash tools/session.sh "ab:hf10M:cur" || exit $?
export VRH_AB='[{"name":"default"},{"name":"waves8","waves_per_simd":8},{"name":"waves8 cap16","waves_per_simd":8,"stack_cap":16}]'
OUT=gpurun_out/s4 bash tools/session.sh "ab:hf10M:cur:primary" || exit $?
export VRH_AB='[{"name":"default"},{"name":"waves6","waves_per_simd":6},{"name":"waves6 cap16","waves_per_simd":6,"stack_cap":16}]'
OUT=gpurun_out/s4 bash tools/session.sh "ab:hf1M:cur" || exit $?
