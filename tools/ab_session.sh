set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out; mkdir -p $OUT
for v in negskip reqconst half both all; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_$v.so timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread \
    "tests/test_gpu_bench_kernel.py::test_benched_step_kernel_vs_oracle[4096-None]" \
    "tests/test_gpu_parity.py::test_batched_reference_rng_vs_oracle_bit_exact" > $OUT/ab_parity_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc $(tail -1 $OUT/ab_parity_$v.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
for r in 1 2 3; do
  for v in sng sng_negskip sng_reqconst sng_half sng_both sng_all; do
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/lib$v.so timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/ab_${r}_$v.log 2>&1 || exit $?
    echo "$r $v $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${r}_$v.log) $(grep -o '"mean_launch_us": [0-9.]*' $OUT/ab_${r}_$v.log)"
  done
done
