#!/bin/bash
# A/B of step-kernel library builds on config 5 (65,536 x 50 x 96, stochastic profiles): parity of each
# build on the wide-kernel tests, then alternating bench runs.  AB_LIBS: library names under lib/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
LIBS="${AB_LIBS:-libsng libsng_w2}"
for l in $LIBS; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
    "tests/test_gpu_wide_kernel.py::test_wide_step_kernel_device_days_vs_oracle_and_general[4096-256]" \
    "tests/test_gpu_lean_sums.py::test_lean_totals_vs_general_kernel_and_oracle[50-True]" \
    "tests/test_gpu_lean_sums.py::test_lean_totals_vs_general_kernel_and_oracle[50-False]" > $OUT/wab_parity_$l.log 2>&1
  rc=$?; echo "parity $l rc=$rc $(tail -1 $OUT/wab_parity_$l.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
for r in 1 2; do
  for l in $LIBS; do
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 python bench.py --no-cpu-baseline --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 8 --warmup 2 > $OUT/wab_${r}_$l.log 2>&1 || exit $?
    echo "$r $l $(grep -o '"ms_per_step": [0-9.]*' $OUT/wab_${r}_$l.log) $(grep -o '"mean_launch_us": [0-9.]*' $OUT/wab_${r}_$l.log) $(grep -o '"eager_launch_us": [0-9.]*' $OUT/wab_${r}_$l.log) $(grep -o '"reset_us": [0-9.]*' $OUT/wab_${r}_$l.log)"
  done
done
