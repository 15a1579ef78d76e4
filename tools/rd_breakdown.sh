#!/bin/bash
# Timing breakdown of ref_day_kernel (reference-RNG day): the product library against diagnostic builds
# without the stream draws (libsng_rdnodraw, -DSNG_RD_NODRAW) and without the timeline stores
# (libsng_rdnostore, -DSNG_RD_NOSTORE), each under rocprofv3 --kernel-trace at 4,096 and 65,536 envs.
#   make -C smart-nanogrid-gym_amd/csrc variants VARIANTS="rdnodraw:-DSNG_RD_NODRAW rdnostore:-DSNG_RD_NOSTORE"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for l in ${RD_LIBS:-libsng libsng_rdnodraw libsng_rdnostore}; do
  SNG_LIBRARY=smart-nanogrid-gym_amd/lib/$l.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/rd_$l \
    -o run --output-format csv -- python tools/reset_bench.py --repeats 3 > gpurun_out/rd_$l.log 2>&1 || exit $?
  python3 - "$l" <<'PY'
import csv, glob, sys
l = sys.argv[1]
f = glob.glob(f"gpurun_out/rd_{l}/**/*kernel_trace.csv", recursive=True)[0]
rows = [x for x in csv.DictReader(open(f)) if "ref_day" in x["Kernel_Name"]]
print(l, [(x["Grid_Size_X"], round((int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000, 1)) for x in rows])
PY
done
