#!/bin/bash
# A/B of library builds on the reference-RNG reset: parity of each build on the reference-RNG tests, then
# tools/reset_bench.py and a kernel-trace of it.  AB_LIBS: library names under lib/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
LIBS="${AB_LIBS:-libsng}"
for l in $LIBS; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -k "golden or batched_reference or many_days or full_size_sampled or config5_extended or sharded" \
    tests/test_gpu_replay.py tests/test_gpu_checkpoint.py tests/test_gpu_recorder.py > $OUT/rab_parity_$l.log 2>&1
  rc=$?; echo "parity $l rc=$rc $(tail -1 $OUT/rab_parity_$l.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
for r in 1 2; do
  for l in $LIBS; do
    SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 python tools/reset_bench.py > $OUT/rab_${r}_$l.log 2>&1 || exit $?
    echo "$r $l $(python -c "import json,sys; [print(d['envs'], round(d['reference_reset']['median_ms'],3), round(d['reference_reset_stream_sync']['median_ms'],3), end='  ') for d in map(json.loads, [x for x in open('$OUT/rab_${r}_$l.log') if x.startswith('{')])]")"
  done
done
for l in $LIBS; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rab_prof_$l -o run --output-format csv -- python tools/reset_bench.py > $OUT/rab_prof_$l.log 2>&1 || exit $?
  grep -E "ref_day|mt_prepare|observe0|py_ratio" $OUT/rab_prof_$l/run_kernel_stats.csv | cut -d, -f1-4
done
