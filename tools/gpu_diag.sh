# Generator / step diagnostics on the GPU box (gpurun -- 'bash tools/gpu_diag.sh'):
#   1. kernel stats of the default build and of a build without hashing, for the generator's floor
#      (hipcc ... -DSNG_GEN_CHEAP -shared -o smart-nanogrid-gym_amd/lib/libsng_gencheap.so
#       sng_kernels.hip sng_api.cpp, in smart-nanogrid-gym_amd/csrc, beforehand);
#   2. one SQ counter pass (8 SQ counters: the per-pass limit) -> tools/sq_summary.py;
#   3. the step kernel at 2 and 4 lanes per env.
# Every GPU step has its own time limit and the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_base -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 8 > $O/base.log 2>&1 || exit $?
SNG_LIBRARY=smart-nanogrid-gym_amd/lib/libsng_gencheap.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_cheap -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 8 > $O/cheap.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR -d $O/sq -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/sq.log 2>&1 || exit $?
for l in 2 4; do timeout -k 10 300 python bench.py --no-cpu-baseline --lanes $l > $O/lanes$l.log 2>&1 || exit $?; done
echo done
