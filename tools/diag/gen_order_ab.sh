#!/bin/bash
# The generator's observation rows dispatched first (the product) or last (tools/diag/patches/
# generator_obs_rows_last.patch -> lib/libsng_obslast.so via tools/diag/variant.sh): same days, order of dispatch.
set -uo pipefail
L=smart-nanogrid-gym_amd/lib
SNG_LIBRARY=$L/libsng.so timeout -k 10 300 python tools/diag/gen_ab_check.py > gpurun_out/order_a.txt 2>&1 || exit 1
SNG_LIBRARY=$L/libsng_obslast.so timeout -k 10 300 python tools/diag/gen_ab_check.py > gpurun_out/order_b.txt 2>&1 || exit 1
diff -q gpurun_out/order_a.txt gpurun_out/order_b.txt > /dev/null && echo "IDENTICAL days" || { echo DIFFER; exit 1; }
for i in 1 2 3; do for v in libsng libsng_obslast; do
 SNG_LIBRARY=$L/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --timing-days 6 > gpurun_out/order_${v}_$i.log 2>&1 || exit 1
 echo "$v $i $(grep -o '"value": [0-9.]*\|"reset_us": [0-9.]*\|"device_ms_per_day": [0-9.]*' gpurun_out/order_${v}_$i.log | head -3 | tr '\n' ' ')"
done; done
