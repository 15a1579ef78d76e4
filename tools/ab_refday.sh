#!/bin/bash
# A/B of reference-RNG days (word / aux / req layouts): tools/reset_bench.py (reference reset, reference day =
# reset + 24 eager steps) with two libraries, alternating, then rocprofv3 kernel stats of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for l in ${AB_LIBS:-libsng libsng_h0 libsng libsng_h0}; do
  i=$((i+1))
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 python tools/reset_bench.py > $OUT/rb${i}_$l.log 2>&1 || exit $?
  echo "rb${i}_$l $(tail -1 $OUT/rb${i}_$l.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: round(d[k]['median_ms'], 4) for k in ('reference_reset_stream_sync', 'reference_reset', 'reference_day', 'device_day')})")"
done
for l in ${PROF_LIBS:-libsng libsng_h0}; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_rb_$l -o run --output-format csv -- python tools/reset_bench.py > $OUT/prof_rb_$l.log 2>&1 || exit $?
done
echo done
