cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_l4w3.so timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_wide_kernel.py > gpurun_out/l4_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/l4_parity.log
if [ $rc -gt 1 ]; then exit $rc; fi
STEPS=ablib AB_LIBS="libsng libsng_l4w3 libsng libsng_l4w3 libsng libsng_l4w3" BENCH_ARGS="--chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 8 --warmup 2" bash tools/gpu_session.sh || exit $?
for f in gpurun_out/ab*_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"reset_us": [0-9.]*' $f) $(grep -o '"mean_launch_us": [0-9.]*' $f)"; done
timeout -k 10 120 rocprofv3 -L > gpurun_out/avail.txt 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVES -d gpurun_out/if5 -o run --output-format csv -- python bench.py --no-cpu-baseline --chargers 50 --time-interval 15min --extended-day --pv-noise 0.2 --price-noise 0.1 --steps 2 --warmup 1 --graph-days 1 --timing-days 1 > gpurun_out/if5.log 2>&1
echo "if5 rc=$?"
