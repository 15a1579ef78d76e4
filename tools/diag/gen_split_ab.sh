#!/bin/bash
# The generator's parts on the headline day (profiles/r06_ab_generator_obs_rows.txt): libsng against two diagnostic
# variants whose days are not valid, built from the current source with tools/diag/variant.sh:
#   g1  no t = 0 observation rows:
#       tools/diag/variant.sh g1 's/(unsigned)(gen_rows(p.n) + (fused ? kObsBlocks : 0))/(unsigned)(gen_rows(p.n))/'
#   g2  the walk computed, its record stores never issued:
#       tools/diag/variant.sh g2 's/        bst16<kGenRecPol>(rec + (size_t)(t + 1) \* nE, el2, occ ? w_occ : w_emp, r2);/        if ((occ ? w_occ : w_emp) == 0x7fffffffu) bst16<kGenRecPol>(rec + (size_t)(t + 1) * nE, el2, occ ? w_occ : w_emp, r2);/'
set -uo pipefail
L=smart-nanogrid-gym_amd/lib
for i in 1 2; do for v in libsng libsng_g1 libsng_g2; do
 SNG_LIBRARY=$L/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --timing-days 6 > gpurun_out/gab_${v}_$i.log 2>&1 || exit 1
 echo "$v $i $(grep -o '"reset_us": [0-9.]*\|"device_ms_per_day": [0-9.]*' gpurun_out/gab_${v}_$i.log | tr '\n' ' ')"
done; done
