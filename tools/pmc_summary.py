"""Summarise rocprofv3 runs of bench.py into profiles/.

  python tools/pmc_summary.py <round-tag> [gpurun_out]

Reads <out>/prof/run_kernel_stats.csv (--kernel-trace --stats) and the two PMC passes
<out>/pmc_fetch/run_counter_collection.csv (FETCH_SIZE) and <out>/pmc_write/... (WRITE_SIZE),
writes profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc.csv and an entry of
profiles/pmc_step_kernel.json; the same for config 5 from prof_cfg5/, pmc5_fetch/ and pmc5_write/
(profiles/<tag>_kernel_stats_config5.csv, profiles/<tag>_pmc_config5.csv).  Every entry carries the build id of
the library measured (<out>/build_id.txt, written by tools/gpu_session.sh; sng_build_id()), and the rocprof
summaries are listed with theirs in profiles/kernel_stats_index.json: bench.py quotes only measurements of the
build it runs.

HBM bytes per launch (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts half the bytes of a coalesced streaming read, so
traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024.  The 2x was checked against this kernel's
own known read volume (the bench's algorithmic read bytes / raw FETCH_SIZE = 1.96).
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    tag = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    build_id = open(os.path.join(out, "build_id.txt")).read().strip()
    meta_path = os.path.join(prof, "pmc_step_kernel.json")
    idx_path = os.path.join(prof, "kernel_stats_index.json")
    try:
        index = json.load(open(idx_path))
    except (OSError, ValueError):
        index = []
    try:
        entries = json.load(open(meta_path))
        entries = entries if isinstance(entries, list) else [entries]
    except (OSError, ValueError):
        entries = []
    # (pass prefix, file suffix, envs, chargers): the headline workload and config 5
    for pre, suf, envs, chargers in (("", "", 65536, 10), ("pmc5_", "_config5", 65536, 50)):
        stats = os.path.join(out, "prof" + ("_cfg5" if suf else ""), "run_kernel_stats.csv")
        fpath = os.path.join(out, (pre or "pmc_") + "fetch", "run_counter_collection.csv")
        wpath = os.path.join(out, (pre or "pmc_") + "write", "run_counter_collection.csv")
        if os.path.exists(stats):
            name = f"profiles/{tag}_kernel_stats{suf}.csv"
            shutil.copyfile(stats, os.path.join(ROOT, name))
            index = [e for e in index if e["file"] != name] + [
                dict(file=name, build_id=build_id, envs=envs, chargers=chargers)]
        if not (os.path.exists(fpath) and os.path.exists(wpath)):
            continue
        fetch, nf = per_kernel(fpath, "FETCH_SIZE")
        write, nw = per_kernel(wpath, "WRITE_SIZE")
        rows = []
        for k in sorted(set(fetch) | set(write)):
            if "sng::" not in k:
                continue
            f, w = fetch.get(k, 0.0), write.get(k, 0.0)
            rows.append(dict(kernel=k.split("(")[0], dispatches=nf.get(k, 0), fetch_kib=round(f, 1),
                             write_kib=round(w, 1), hbm_bytes_per_launch=int(2 * f * 1024 + w * 1024)))
        with open(os.path.join(prof, f"{tag}_pmc{suf}.csv"), "w", newline="") as fp:
            wr = csv.DictWriter(fp, fieldnames=list(rows[0]))
            wr.writeheader()
            wr.writerows(rows)
        step = [r for r in rows if "step_" in r["kernel"]][0]
        meta = dict(source=f"profiles/{tag}_pmc{suf}.csv (rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes)",
                    build_id=build_id, kernel=step["kernel"], envs=envs, chargers=chargers, bytes_per_launch=step["hbm_bytes_per_launch"],
                    fetch_kib=step["fetch_kib"], write_kib=step["write_kib"],
                    correction="traffic = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE counts half of streamed reads)")
        entries = [e for e in entries if not (e.get("envs") == envs and e.get("chargers") == chargers
                                              and e.get("build_id") == build_id)] + [meta]
        for r in rows:
            print(r)
    json.dump(entries, open(meta_path, "w"), indent=1)
    json.dump(index, open(idx_path, "w"), indent=1)


if __name__ == "__main__":
    main()
