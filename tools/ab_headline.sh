#!/bin/bash
# A/B of library builds on the headline config (65,536 x 10 x 24): parity of each build on the benched
# kernel's oracle test, then alternating bench runs.  AB_LIBS: library names under lib/; AB_ROUNDS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
LIBS="${AB_LIBS:-libsng}"
for l in $LIBS; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
    "tests/test_gpu_bench_kernel.py::test_benched_step_kernel_vs_oracle[4096-None]" ${AB_TESTS:-} > $OUT/hab_parity_$l.log 2>&1
  rc=$?; echo "parity $l rc=$rc $(tail -1 $OUT/hab_parity_$l.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
for r in $(seq 1 ${AB_ROUNDS:-3}); do
  for l in $LIBS; do
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/hab_${r}_$l.log 2>&1 || exit $?
    echo "$r $l $(grep -o '"ms_per_step": [0-9.]*' $OUT/hab_${r}_$l.log) $(grep -o '"mean_launch_us": [0-9.]*' $OUT/hab_${r}_$l.log) $(grep -o '"eager_launch_us": [0-9.]*' $OUT/hab_${r}_$l.log) $(grep -o '"reset_us": [0-9.]*' $OUT/hab_${r}_$l.log)"
  done
done
