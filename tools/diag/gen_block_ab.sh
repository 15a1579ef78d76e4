#!/bin/bash
# The generator's workgroup size (kGenBlock: 256 in the product; variants libsng_gb128 / libsng_gb512 built with
# tools/diag/variant.sh 's/^constexpr int kGenBlock = 256; /constexpr int kGenBlock = 128; /' and 512): the same
# days (gen_ab_check.py), then the headline day.
set -uo pipefail
L=smart-nanogrid-gym_amd/lib
for v in libsng libsng_gb128 libsng_gb512; do
 SNG_LIBRARY=$L/$v.so timeout -k 10 300 python tools/diag/gen_ab_check.py > gpurun_out/gb_$v.txt 2>&1 || { tail -3 gpurun_out/gb_$v.txt; exit 1; }
done
for v in libsng_gb128 libsng_gb512; do diff -q gpurun_out/gb_libsng.txt gpurun_out/gb_$v.txt > /dev/null && echo "$v: identical days" || { echo "$v: DIFFER"; exit 1; }; done
for i in 1 2 3; do for v in libsng libsng_gb128 libsng_gb512; do
 SNG_LIBRARY=$L/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --timing-days 6 > gpurun_out/gb_${v}_$i.log 2>&1 || exit 1
 echo "$v $i $(grep -o '"value": [0-9.]*\|"reset_us": [0-9.]*\|"device_ms_per_day": [0-9.]*' gpurun_out/gb_${v}_$i.log | head -3 | tr '\n' ' ')"
done; done
