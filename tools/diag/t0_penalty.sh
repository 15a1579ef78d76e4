#!/bin/bash
# Why are a day's first two steps ~0.7 us slower in the graph (profiles/r06b_trace_split.txt)?  Per-timestep step
# times from a kernel trace of the bench, for the product and for variants (LIBS, built with tools/diag/variant.sh).
set -uo pipefail
export TMPDIR=/tmp
L=smart-nanogrid-gym_amd/lib
for v in ${LIBS:-libsng libsng_recpol}; do
 rm -rf gpurun_out/t0_$v
 SNG_LIBRARY=$L/$v.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/t0_$v -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/t0_$v.log 2>&1 || exit 1
 echo "== $v"; python tools/trace_split.py gpurun_out/t0_$v/run_kernel_trace.csv 2>&1 | grep "graph"
done
