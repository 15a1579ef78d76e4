#!/bin/bash
# The step kernel's workgroup -> env mapping: consecutive workgroups (the product) or XCD-contiguous env ranges
# (workgroup i runs on XCD i mod 8: libsng_xcd, built with tools/diag/variant.sh on step_wide_kernel's e0 line).
set -uo pipefail
L=smart-nanogrid-gym_amd/lib
for i in 1 2 3; do for v in libsng libsng_xcd; do
 SNG_LIBRARY=$L/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/xcd_${v}_$i.log 2>&1 || exit 1
 echo "$v $i $(grep -o '"value": [0-9.]*\|"mean_launch_us": [0-9.]*\|"eager_launch_us": [0-9.]*\|"device_ms_per_day": [0-9.]*' gpurun_out/xcd_${v}_$i.log | head -4 | tr '\n' ' ')"
done; done
