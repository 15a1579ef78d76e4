#!/bin/bash
# A/B of the wide step kernel's scheduling groups (SNG_WIDE_SB: chargers between sched_barriers): parity of
# each variant on the wide and benched kernels' oracle tests, then alternating config-5 and headline benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V="${SB_LIBS:-libsng_sb2 libsng_sb5 libsng_sb25}"
for l in $V; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
    tests/test_gpu_wide_kernel.py "tests/test_gpu_bench_kernel.py::test_benched_step_kernel_vs_oracle[4096-None]" > gpurun_out/par_$l.log 2>&1
  rc=$?; echo "parity $l rc=$rc $(tail -1 gpurun_out/par_$l.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
C5="--chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 8 --warmup 2"
for r in 1 2; do
  for l in libsng $V; do
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 python bench.py --no-cpu-baseline $C5 > gpurun_out/c5_${r}_$l.log 2>&1 || exit $?
    echo "c5 $r $l $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c5_${r}_$l.log) $(grep -o '"mean_launch_us": [0-9.]*' gpurun_out/c5_${r}_$l.log)"
  done
done
for r in 1 2; do
  for l in libsng $V; do
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/h_${r}_$l.log 2>&1 || exit $?
    echo "h $r $l $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/h_${r}_$l.log) $(grep -o '"mean_launch_us": [0-9.]*' gpurun_out/h_${r}_$l.log)"
  done
done
