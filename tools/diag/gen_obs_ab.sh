#!/bin/bash
# A generator rewrite against the build before it (profiles/r06_ab_generator_obs_rows.txt): copy the old library to
# lib/libsng_base.so, build the new one as lib/libsng.so (e.g. with tools/diag/patches/generator_obs_in_timeline.patch
# applied), then: every device day must hash the same (tools/diag/gen_ab_check.py), and the bench A/B follows.
set -uo pipefail
L=smart-nanogrid-gym_amd/lib
SNG_LIBRARY=$L/libsng_base.so timeout -k 10 300 python tools/diag/gen_ab_check.py > gpurun_out/genobs_a.txt 2>&1 || { tail -5 gpurun_out/genobs_a.txt; exit 1; }
timeout -k 10 300 python tools/diag/gen_ab_check.py > gpurun_out/genobs_b.txt 2>&1 || { tail -5 gpurun_out/genobs_b.txt; exit 1; }
if diff gpurun_out/genobs_a.txt gpurun_out/genobs_b.txt > gpurun_out/genobs_diff.txt; then echo "IDENTICAL $(wc -l < gpurun_out/genobs_a.txt) lines"; else echo "DIFFER"; head -20 gpurun_out/genobs_diff.txt; exit 1; fi
for i in 1 2; do for v in libsng_base libsng; do
 SNG_LIBRARY=$L/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --timing-days 6 > gpurun_out/genobs_${v}_$i.log 2>&1 || exit 1
 echo "$v $i $(grep -o '"value": [0-9.]*\|"reset_us": [0-9.]*\|"device_ms_per_day": [0-9.]*\|"mean_launch_us": [0-9.]*' gpurun_out/genobs_${v}_$i.log | tr '\n' ' ')"
done; done
