set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out; mkdir -p $OUT
for l in libsng libsng_rdnoph1 libsng_rdnostore libsng_rde32 libsng_rde16; do
  for envs in 65536 4096; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/rd_${l}_${envs}p -o run --output-format csv -- python tools/reset_bench.py --envs $envs > $OUT/rd_${l}_$envs.log 2>&1 || exit $?
  echo "$l $envs $(grep -E 'ref_day' $OUT/rd_${l}_${envs}p/run_kernel_stats.csv | cut -d, -f2-4) ref_reset_ms=$(python -c "import json; print([round(json.loads(x)['reference_reset']['median_ms'],3) for x in open('$OUT/rd_${l}_$envs.log') if x.startswith('{')])")"
  done
done
