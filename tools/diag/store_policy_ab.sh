#!/bin/bash
# A/B of the state stores' cache policy (SoC pairs, BESS, day return, flags: bst / bst2 in sng_kernels.hip) on the
# headline day: libsng (nt), libsng_wt (sc0 | sc1 | nt: written through at system scope), libsng_wt1 (sc0 | sc1),
# built by tools/diag/variant.sh.  Why: without an agent-scope release a next kernel on another XCD reads stale
# lines (profiles/r06_coherence_probe.txt), so every step ends with an L2 writeback of what it left dirty.
set -uo pipefail
L=smart-nanogrid-gym_amd/lib
for i in 1 2; do for v in ${LIBS:-libsng libsng_wt libsng_wt1}; do
 SNG_LIBRARY=$L/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/stpol_${v}_$i.log 2>&1 || exit 1
 echo "$v $i $(grep -o '"value": [0-9.]*\|"reset_us": [0-9.]*\|"device_ms_per_day": [0-9.]*\|"mean_launch_us": [0-9.]*\|"eager_launch_us": [0-9.]*' gpurun_out/stpol_${v}_$i.log | tr '\n' ' ')"
done; done
