set -uo pipefail
L=smart-nanogrid-gym_amd/lib
for i in 1 2; do for v in libsng libsng_g1 libsng_g2; do
 SNG_LIBRARY=$L/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --timing-days 6 > gpurun_out/gab_${v}_$i.log 2>&1 || exit 1
 echo "$v $i $(grep -o '"reset_us": [0-9.]*\|"device_ms_per_day": [0-9.]*' gpurun_out/gab_${v}_$i.log | tr '\n' ' ')"
done; done
