#!/bin/bash
# Does the length of the untimed warm-up move the headline?  bench.py --no-cpu-baseline with warm-ups of 8 (the
# default), 200 and 2,000 days, interleaved, on one box.
set -uo pipefail
for i in 1 2 3; do for w in 8 200 2000; do
 timeout -k 10 180 python bench.py --no-cpu-baseline --warmup $w > gpurun_out/warm_${w}_$i.log 2>&1 || exit 1
 echo "warmup $w run $i $(grep -o '"value": [0-9.]*\|"device_ms_per_day": [0-9.]*\|"mean_launch_us": [0-9.]*' gpurun_out/warm_${w}_$i.log | head -3 | tr '\n' ' ')"
done; done
