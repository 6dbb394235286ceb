#!/bin/bash
# One parametrized GPU session (replaces the per-round session scripts of rounds 2-4).
#   OUT=gpurun_out/<dir> tools/session.sh STEP [STEP ...]
# Steps (each with its own time limit; a fault / abort / timeout ends the session):
#   tests[:K]        pytest -m gpu (optionally -k K)          smoke       __graft_entry__.smoke()
#   bench:<cfg>      the driver's shape (--steps 20 --warmup 5) on cfg = c3 (with the CPU baseline and
#                    the user-kernel leg) | c4 | c2 | c5 | f32 (the no-argument command) | shards8
#   pmc:<cfg>        TCP / HBM read / HBM write counter passes of bench:<cfg> and their summary
#                    (tools/pmc_bench.py -> profiles/pmc_traffic_F<F>[_<scene>_<kernel>].json)
#   mem:<cfg>        L2 hit / TD busy / TD stall passes of bench:<cfg>
#   trace:<cfg>      rocprofv3 --kernel-trace --stats of bench:<cfg>
#   ab:<scene>:<libs>[:<kernel>]   same-box A/B of library builds (tools/ab_builds.sh), libs comma-separated
#   pmcuser:<lambda|defer|ref>  trace + counter passes of a user-kernel program (32 frames per launch, C3) and
#                    their summary (tools/pmc_user.py -> profiles/pmc_user_<lambda|ref>.json)
#   user[:reps]      user-kernel throughput: AO lambda and ao/main.cpp's kernel, 1 and 32 frames per launch
#   counters         rocprofv3 -L (the counters this box offers)
#   cmd:<name>:<seconds>:<command> anything else
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/session}
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  tail -${TAIL:-2} $OUT/$name.log | cut -c1-400; echo "$name rc=$rc"
  if fatal $rc; then echo "fatal exit; stopping"; exit $rc; fi
  [ $rc = 0 ] || exit $rc
}
Q="--no-cpu-baseline --single-frames 0 --moving-camera 0 --no-user-kernel --no-verify"
cfg_args() {  # cfg -> bench arguments (driver shape)
  case $1 in
    c3) echo "--steps 20 --warmup 5";;
    c4) echo "--scene hf10M --steps 20 --warmup 5";;
    c2) echo "--scene hf1M --kernel primary --steps 20 --warmup 5";;
    c5) echo "--scene sph1M --steps 20 --warmup 5";;
    f32) echo "";;
    shards8) echo "--steps 20 --warmup 5 --shards 8";;
    *) echo "unknown cfg $1" >&2; exit 2;;
  esac
}
cfg_meta() {  # cfg -> scene kernel F
  case $1 in c3) echo "hf1M ao 20";; c4) echo "hf10M ao 20";; c2) echo "hf1M primary 20";;
             c5) echo "sph1M primary 20";; f32) echo "hf1M ao 32";; esac
}
n_tests=0
for s in "$@"; do
  kind=${s%%:*}; arg=${s#*:}; [ "$arg" = "$s" ] && arg=
  case $kind in
    tests) n_tests=$((n_tests + 1)); TAIL=4 step pytest_gpu_$n_tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 \
             --timeout-method thread ${arg:+-k "$arg"};;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    bench) extra="--no-cpu-baseline"; [ "$arg" = c3 ] && extra=""
           step bench_$arg 600 python3 bench.py $(cfg_args $arg) $extra;;
    pmc)   a="$(cfg_args $arg) $Q"; set -- $(cfg_meta $arg); sc=$1 kn=$2 F=$3; d=$OUT/pmc_$arg
           step pmc_${arg}_tcp 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD --output-format csv -d $d/pmc_bench_tcp -o run -- python3 bench.py $a
           step pmc_${arg}_hbm 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/pmc_bench_hbm -o run -- python3 bench.py $a
           step pmc_${arg}_wr 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/pmc_bench_wr -o run -- python3 bench.py $a
           name=pmc_traffic_F$F.json; [ "$arg" != c3 ] && [ "$arg" != f32 ] && name=pmc_traffic_F${F}_${sc}_${kn}.json
           python3 tools/pmc_bench.py $d $d/$name $sc $kn $F "python3 bench.py $a" && cp $d/$name profiles/;;
    mem)   a="$(cfg_args $arg) $Q"; d=$OUT/mem_$arg
           step mem_${arg}_tcc 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $d/tcc -o run -- python3 bench.py $a
           step mem_${arg}_td 300 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE --output-format csv -d $d/td -o run -- python3 bench.py $a;;
    trace) step trace_$arg 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$arg -o run -- python3 bench.py $(cfg_args $arg) --no-cpu-baseline;;
    ab)    IFS=: read -r sc libs kn <<< "$arg"
           LIBS="${libs//,/ }" SCENES=$sc KERNEL=${kn:-ao} step ab_${sc}_${kn:-ao} 900 bash tools/ab_builds.sh;;
    pmcuser) # lambda: the restated AO lambda (bench's user leg), defer: the same with deferred any_hit
             # calls (VRH_USER_DEFER), ref: ao/main.cpp's own kernel through the reference's headers -- all on
             # hip_sched::frames, 32 frames per launch, C3
           case $arg in lambda) prog="build/tests/user_kernels bench 708 1920 1080 /tmp 4 32";;
                        defer) prog="build/tests/uk_defer bench 708 1920 1080 /tmp 4 32";;
                        ref) prog="oracle/_ref/ref_kernels bench hf1M 1920 1080 4 32";; esac
           d=$OUT/pmcuser_$arg
           step pmcuser_${arg}_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- $prog
           step pmcuser_${arg}_tcp 300 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD --output-format csv -d $d/pmc_tcp -o run -- $prog
           step pmcuser_${arg}_hbm 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/pmc_hbm -o run -- $prog
           step pmcuser_${arg}_wr 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/pmc_wr -o run -- $prog
           step pmcuser_${arg}_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $d/pmc_sq -o run -- $prog
           python3 tools/pmc_user.py $d $d/pmc_user_$arg.json "$prog" 32 $d/trace && cp $d/pmc_user_$arg.json profiles/;;
    user)  # user-kernel throughput (C3): the restated AO lambda and ao/main.cpp's own kernel (reference
           # headers), one frame per launch and 32 in flight, alternating, ${arg:-2} repetitions
           for rep in $(seq 1 ${arg:-2}); do for F in ${FS:-1 32}; do L=20; [ $F -gt 1 ] && L=4
             for b in ${BINS:-build/tests/user_kernels build/tests/uk_defer oracle/_ref/ref_kernels oracle/_ref/ref_kernels_defer}; do [ -x $b ] || continue
               case $b in *ref_kernels*) a="bench hf1M 1920 1080 $L $F";; *) a="bench 708 1920 1080 /tmp $L $F";; esac
               TAIL=1 step user_$(basename $b)_F${F}_$rep 150 $b $a
               echo "$(basename $b) F=$F $(grep frame_ms_median $OUT/user_$(basename $b)_F${F}_$rep.log)" >> $OUT/user.log
             done; done; done;;
    sq)    # one SQ pass (VALU lane utilisation, instructions per ray, issue / wait shares, waves):
           # sq:<cfg> the built-in kernel of bench:<cfg> (RAYS = its rays per frame, default C3's),
           # sq:lambda / sq:ref the user-kernel programs
           SQC="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU"
           d=$OUT/sq_$arg
           case $arg in
             lambda) step sq_$arg 300 rocprofv3 --pmc $SQC --output-format csv -d $d -o run -- build/tests/user_kernels bench 708 1920 1080 /tmp 4 32
                     python3 tools/pmc_sq.py $d $d/pmc_sq_$arg.json "$arg" 32 13037200 user_render;;
             uk_*)   step sq_$arg 300 rocprofv3 --pmc $SQC --output-format csv -d $d -o run -- build/tests/$arg bench 708 1920 1080 /tmp 4 32
                     python3 tools/pmc_sq.py $d $d/pmc_sq_$arg.json "$arg" 32 13037200 user_render;;
             ref)    step sq_$arg 300 rocprofv3 --pmc $SQC --output-format csv -d $d -o run -- oracle/_ref/ref_kernels bench hf1M 1920 1080 4 32
                     python3 tools/pmc_sq.py $d $d/pmc_sq_$arg.json "$arg" 32 13037200 user_render;;
             *)      a="$(cfg_args $arg) $Q"; set -- $(cfg_meta $arg)
                     step sq_$arg 300 rocprofv3 --pmc $SQC --output-format csv -d $d -o run -- python3 bench.py $a
                     python3 tools/pmc_sq.py $d $d/pmc_sq_$arg.json "$arg" $3 ${RAYS:-13037200};;
           esac;;
    counters) step counters_list 120 rocprofv3 -L;;
    cmd)   IFS=: read -r name t c <<< "$arg"; step $name $t bash -c "$c";;
    *) echo "unknown step $s"; exit 2;;
  esac
done
exit 0
