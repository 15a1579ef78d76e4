#!/bin/bash
# A/B of the packet chain against the hipGraph (the headline day in the bench, 100 days, interleaved rounds).
# Needs the chain: apply tools/diag/patches/aql_packet_chain.patch (bench.py --dispatch aql) and rebuild.
# Results: profiles/r06_ab_packet_chain.txt.
# Configurations: SNG_AQL_FENCES (a = agent, n = none; acquire then release), SNG_AQL_NO_STREAM_WAIT (the caller's
# stream does not wait for the chain: HIP runs that wait as a polling kernel), SNG_AQL_DIMS3 (HIP's 3-dimension
# setup).  HIP's own packets carry acquire agent / release agent (tools/diag/hip_header_probe.hip).
set -uo pipefail
CFGS=${CFGS:-graph aa aa_nowait aa_dims3_nowait}
for i in 1 2; do
 for cfg in $CFGS; do
  env_=(SNG_AQL_FENCES=aa); d=aql
  case $cfg in
   graph) d=graph ;;
   an) env_=(SNG_AQL_FENCES=an) ;;
   aa_nowait) env_+=(SNG_AQL_NO_STREAM_WAIT=1) ;;
   aa_dims3_nowait) env_+=(SNG_AQL_NO_STREAM_WAIT=1 SNG_AQL_DIMS3=1) ;;
   aa_dims3) env_+=(SNG_AQL_DIMS3=1) ;;
   aa_fine) env_+=(SNG_AQL_FINE_KERNARG=1) ;;
  esac
  env "${env_[@]}" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 100 --warmup 10 --dispatch $d > gpurun_out/ab_${cfg}_${i}.log 2>&1 || exit 1
  echo "$cfg $i $(grep -o '"value": [0-9.]*\|"device_ms_per_day": [0-9.]*\|"mean_launch_us": [0-9.]*' gpurun_out/ab_${cfg}_${i}.log | tr '\n' ' ')"
 done
done
