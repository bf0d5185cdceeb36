#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run into profiles/<tag>_*.

  python tools/pmc_traffic.py <tag> [kernel-substring] [bench-kernel-name]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats of the bench command),
profiles/<tag>_bench.json (the bench line) and profiles/<tag>_traffic.json:
per-launch HBM bytes of the dominant kernel from the separate FETCH_SIZE and
WRITE_SIZE passes, corrected as MI355X_MICROARCH.md §HBM prescribes
(counters in KiB; FETCH_SIZE reads half the bytes of a wide coalesced stream on
gfx950 -> x2), averaged over the same launch mix bench.py times.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def per_launch(path, counter, sub):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and sub in r["Kernel_Name"]]
    return (sum(vals) / len(vals) if vals else None), len(vals)


def main():
    tag = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "Conv2Dgrad"
    bench_kernel = sys.argv[3] if len(sys.argv) > 3 else "conv2_dgrad"
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(OUT, "prof", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    line = [l for l in open(os.path.join(OUT, "bench_full.log")) if l.startswith("{")][-1]
    open(os.path.join(prof, f"{tag}_bench.json"), "w").write(line)
    fetch, nf = per_launch(os.path.join(OUT, "pmcb", "fetch_counter_collection.csv"), "FETCH_SIZE", sub)
    write, nw = per_launch(os.path.join(OUT, "pmcb", "write_counter_collection.csv"), "WRITE_SIZE", sub)
    avg_ms = None
    for r in csv.DictReader(open(os.path.join(OUT, "prof", "run_kernel_stats.csv"))):
        if sub in r["Name"]:
            avg_ms = float(r["AverageNs"]) / 1e6
            calls = int(r["Calls"])
    rd = 2.0 * fetch * 1024
    wr = write * 1024
    out = {"kernel": bench_kernel, "kernel_match": sub, "launches_fetch_pass": nf, "launches_write_pass": nw,
           "fetch_bytes_per_launch": rd, "write_bytes_per_launch": wr, "traffic_bytes_per_launch": rd + wr,
           "rocprof_avg_launch_ms": avg_ms, "rocprof_calls": calls,
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count of wide streaming reads), WRITE_SIZE KiB x1024",
           "source": "tools/profile_round.sh: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) of "
                     "`python3 bench.py --no-cpu-baseline --no-gae-roofline`"}
    out["tag"] = tag
    out["workload"] = json.loads(line)["config"]["workload"]   # bench.py only uses traffic of the same workload
    json.dump(out, open(os.path.join(prof, f"{tag}_traffic.json"), "w"), indent=1)
    # the file bench.py reads to fill roofline.traffic for this kernel
    json.dump(out, open(os.path.join(prof, "roofline_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
