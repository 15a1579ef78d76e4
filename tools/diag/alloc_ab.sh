#!/bin/bash
# A/B of the state's memory type (tools/diag/patches/state_alloc_flags.patch -> lib/libsng_allocfl.so):
# hipMalloc (the product), hipDeviceMallocUncached for every state array / all but the timeline planes / only
# those, hipDeviceMallocFinegrained, on the headline day.
set -uo pipefail
L=smart-nanogrid-gym_amd/lib
for i in 1 2; do
 for cfg in ${CFGS:-base uncached uncached_state uncached_timeline}; do
  case $cfg in
   base) env_=(SNG_LIBRARY=$L/libsng.so) ;;
   *) env_=(SNG_LIBRARY=$L/libsng_allocfl.so SNG_ALLOC_FLAGS=$cfg) ;;
  esac
  env "${env_[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/alloc_${cfg}_${i}.log 2>&1 || exit 1
  echo "$cfg $i $(grep -o '"value": [0-9.]*\|"device_ms_per_day": [0-9.]*\|"mean_launch_us": [0-9.]*\|"reset_us": [0-9.]*' gpurun_out/alloc_${cfg}_${i}.log | tr '\n' ' ')"
 done
done
