#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel stats.  Every GPU step has its own time
# limit; the script stops at the first fatal exit (abort/segfault/timeout), and continues past
# ordinary test failures (exit 1) so the bench still runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # run <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session.log
  timeout -k 10 "$to" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session.log
  tail -5 $OUT/$name.log | tee -a $OUT/session.log
  if fatal $rc; then echo "fatal exit $rc in $name; stopping" | tee -a $OUT/session.log; exit $rc; fi
  return 0
}
# the build id of the library the session measures (profiles/ are keyed by it: tools/pmc_summary.py, bench.py)
python -c "import sys; sys.path.insert(0, 'smart-nanogrid-gym_amd'); from smart_nanogrid_gym import _native; print(_native.lib().sng_build_id().decode())" > $OUT/build_id.txt
echo "=== build id $(cat $OUT/build_id.txt)" | tee -a $OUT/session.log
STEPS="${STEPS:-tests smoke bench prof}"
for s in $STEPS; do
  case $s in
    tests) if [ -n "${PYTEST_K:-}" ]; then run pytest_gpu 1100 python -u -m pytest tests -m gpu -q -ra --timeout 300 --timeout-method thread -k "$PYTEST_K"
           else run pytest_gpu 1100 python -u -m pytest tests -m gpu -q -ra --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}; fi ;;
    one)   run pytest_one 600 python -m pytest ${ONE_TESTS:-tests/test_gpu_recorder.py} -m gpu -q ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    ablib|ablib2) tag=${s/ablib/ab}; args=${BENCH_ARGS:-}; [ $s = ablib2 ] && args=${BENCH_ARGS2:-}
           i=0; for l in ${AB_LIBS:?AB_LIBS="libsng_<name> libsng ..." (tools/diag/variant.sh)}; do i=$((i+1)); SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so run "${tag}-${i}_$l" 300 python bench.py --no-cpu-baseline $args; done
           for f in $OUT/${tag}-*_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"mean_launch_us": [0-9.]*' $f)"; done | tee -a $OUT/session.log ;;
    ab)    for a in ${AB_ARGS:-"--pipeline 0" "--pipeline 1"}; do run "bench_ab_${a// /_}" 300 python bench.py --no-cpu-baseline $a; done ;;
    sweep) for l in 1 2 4; do run bench_l$l 300 python bench.py --no-cpu-baseline --lanes $l; done ;;
    v2x)   run bench_v2x 300 python bench.py --no-cpu-baseline --v2x --steps 40
           run bench_v2x50 300 python bench.py --no-cpu-baseline --v2x --chargers 50 --steps 10 --graph-days 5 ;;
    sq)    for l in ${SQ_LANES:-1 2}; do run sq_l$l 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/sq_l$l -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 --lanes $l; done ;;
    sqw)   run sq_wide 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d $OUT/sq_wide -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1
           run sq_wide5 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU -d $OUT/sq_wide5 -o run --output-format csv -- python bench.py --no-cpu-baseline --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 2 --warmup 1 --graph-days 1 --timing-days 1 ;;
    stamps) SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_stamps.so run stamps 300 python tools/stamps.py ;;
    rdstamps) for l in ${RD_LIBS:-libsng_stamps}; do SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so run "rdstamps_$l" 300 python tools/rd_stamps.py; done ;;
    prof)  run prof_stats 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --no-cpu-baseline ;;
    cfg5)  run bench_cfg5 600 python bench.py --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 8 --warmup 2 --cpu-budget 12
           run prof_cfg5 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_cfg5 -o run --output-format csv -- python bench.py --no-cpu-baseline --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 8 --warmup 2 ;;
    closed) run closed_loop 600 python tools/closed_loop_bench.py
            run closed_loop_mlp 600 python tools/closed_loop_bench.py --policy mlp ;;
    memfloor) SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_memfloor.so run memfloor 300 python bench.py --no-cpu-baseline
           SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_memfloor.so run memfloor_cfg5 300 python bench.py --no-cpu-baseline --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 8 --warmup 2 ;;
    reset) run reset_bench 600 python tools/reset_bench.py ;;
    resetab) i=0; for l in ${RESET_LIBS:?RESET_LIBS="libsng_<name> libsng ..."}; do i=$((i+1)); SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so run "reset${i}_$l" 300 python tools/reset_bench.py --envs 65536; done ;;
    resetprof) run reset_prof 600 rocprofv3 --kernel-trace --stats -d $OUT/reset_prof -o run --output-format csv -- python tools/reset_bench.py --envs 65536 ;;
    layout) run stepmem2 300 tools/stepmem2 ;;
    goverhead) run graph_overhead 300 tools/graph_overhead ;;
    sb3ab) for i in 1 2; do SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng.so run "sb3_old$i" 300 python tools/sb3_path_bench.py --pkg tools/diag/old_pkg
                            run "sb3_new$i" 300 python tools/sb3_path_bench.py; done
           run host_copy 120 python tools/host_copy_bench.py ;;
    single) run single_env_host 300 python tools/single_env_bench.py
            run single_env_torch 300 python tools/single_env_bench.py --path torch
            run single_env_device 300 python tools/single_env_bench.py --rng device ;;
    iolat) run io_latency 120 tools/io_latency ;;
    overlap) run overlap_probe 300 python tools/overlap_probe.py ;;
    genab) for l in ${AB_LIBS:?}; do SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so run "genab_$l" 300 python tools/diag/gen_ab_check.py; done
           set -- ${AB_LIBS}; if diff <(grep '^E=' $OUT/genab_$1.log) <(grep '^E=' $OUT/genab_$2.log) > $OUT/genab_diff.txt; then echo "genab: identical" | tee -a $OUT/session.log; else echo "genab: DIFFER" | tee -a $OUT/session.log; fi ;;
    sqsalu) for l in ${SQ_LIBS:-libsng}; do SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so run "sqsalu_$l" 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/sqsalu_$l -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1; done ;;
    sb3c)  run sb3_consume 600 python tools/sb3_path_bench.py --consume ;;
    sb3)   run sb3_path 600 python tools/sb3_path_bench.py
           run sb3_path_device 600 python tools/sb3_path_bench.py --rng device ;;
    pmc5)  run pmc5_fetch 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc5_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 2 --warmup 1 --graph-days 1 --timing-days 1
           run pmc5_write 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc5_write -o run --output-format csv -- python bench.py --no-cpu-baseline --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 2 --warmup 1 --graph-days 1 --timing-days 1 ;;
    pmc)   run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1
           run pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 ;;
  esac
done
echo "=== session done" | tee -a $OUT/session.log
