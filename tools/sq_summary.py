"""Per-kernel means of every counter in rocprofv3 counter_collection CSVs.

  python tools/sq_summary.py gpurun_out/sq_l1/run_counter_collection.csv [...]
"""
import collections
import csv
import sys

for path in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(path)
    for k, cs in agg.items():
        if "sng::" not in k:
            continue
        print(" ", k, {c: round(sum(v) / len(v), 1) for c, v in sorted(cs.items())})
