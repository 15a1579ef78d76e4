#!/bin/bash
# HIP runtime knobs against the headline day (never changes the library): each configuration runs the bench
# twice, interleaved, under its own time limit; the JSON lines land in gpurun_out/knobs/<name>_<i>.log.
# ROC_SYSTEM_SCOPE_SIGNAL=0 is left out: its bench hung until its time limit (profiles/r06_ab_hip_env_knobs.txt).
#   tools/gpu ... -- 'bash tools/diag/env_knobs.sh'
set -uo pipefail
mkdir -p gpurun_out/knobs
configs=(
  "base:"
  "pc0:DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"
  "pc1:DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"
  "hdp0:DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0"
  "hdp1:DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1"
  "dd0:AMD_DIRECT_DISPATCH=0"
  "dk0:HIP_FORCE_DEV_KERNARG=0"
  "skip1:ROC_SKIP_KERNEL_ARG_COPY=1"
)
for i in 1 2; do
  for c in "${configs[@]}"; do
    name=${c%%:*}; kv=${c#*:}
    if [ -n "$kv" ]; then
      env "$kv" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "gpurun_out/knobs/${name}_$i.log" 2>&1
    else
      timeout -k 10 120 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "gpurun_out/knobs/${name}_$i.log" 2>&1
    fi
    rc=$?
    echo "$name $i rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python - <<'PY'
import glob, json, os
rows = {}
for f in sorted(glob.glob("gpurun_out/knobs/*.log")):
    name = os.path.basename(f)[:-4].rsplit("_", 1)[0]
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            r = d["roofline"]
            rows.setdefault(name, []).append((round(d["value"] / 1e9, 3), r["device_ms_per_day"], r["mean_launch_us"], r["reset_us"]))
for k, v in rows.items():
    print(k, v)
PY
