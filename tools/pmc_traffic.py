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


def mfma_util(path):
    """per kernel name: average MFMA pipeline utilisation over its launches"""
    if not os.path.exists(path):
        return None
    per, dur = {}, {}
    for r in csv.DictReader(open(path)):
        key = (r["Kernel_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))
        per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            dur[key] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    agg = {}
    for key, c in per.items():
        if "GRBM_GUI_ACTIVE" not in c or "SQ_VALU_MFMA_BUSY_CYCLES" not in c or c["GRBM_GUI_ACTIVE"] <= 0:
            continue
        short = key[0].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:80]
        a = agg.setdefault(short, [0, 0.0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        a[2] += c["GRBM_GUI_ACTIVE"]
        a[3] += c.get("SQ_INSTS_MFMA", 0.0)
        a[4] += dur.get(key, 0.0)
    out = {}
    for k, (n, busy, gui, insts, ns) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        if insts <= 0:
            continue
        out[k] = {"launches": n, "mfma_util": round(busy / (1024 * gui / 8), 4), "mfma_insts_per_launch": insts / n}
        if ns > 0:
            # the shader clock the kernel ran at: GRBM_GUI_ACTIVE counts GPU-busy
            # cycles summed over the 8 XCDs, over the same dispatches' durations
            out[k]["sclk_ghz"] = round(gui / 8 / ns, 4)
            out[k]["pmc_avg_launch_ms"] = round(ns / n / 1e6, 4)
    return out


def main():
    tag = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "Conv2Dgrad"
    bench_kernel = sys.argv[3] if len(sys.argv) > 3 else "conv2_dgrad"
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(OUT, "prof", "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    line = [l for l in open(os.path.join(OUT, "bench_full.log")) if l.startswith("{")][-1]
    open(os.path.join(prof, f"{tag}_bench.json"), "w").write(line)
    # sub may name several kernels ("a|b"): one bench launch that runs them in
    # sequence (conv2 forward: the five-tile kernel + the lone-pixel kernel); the
    # per-launch figures are then the sums of the parts' per-launch averages
    fetch = write = 0.0
    nf = nw = 0
    avg_ms = 0.0
    calls = 0
    for part in sub.split("|"):
        f, n1 = per_launch(os.path.join(OUT, "pmcb", "fetch_counter_collection.csv"), "FETCH_SIZE", part)
        w, n2 = per_launch(os.path.join(OUT, "pmcb", "write_counter_collection.csv"), "WRITE_SIZE", part)
        fetch += f or 0.0
        write += w or 0.0
        nf, nw = max(nf, n1), max(nw, n2)
        # every instantiation of the kernel (e.g. the rollout and the mask-writing
        # training forward) together: the launch mix bench.py's events time
        tot_ns, c = 0.0, 0
        for r in csv.DictReader(open(os.path.join(OUT, "prof", "run_kernel_stats.csv"))):
            if part in r["Name"]:
                tot_ns += float(r["TotalDurationNs"])
                c += int(r["Calls"])
        avg_ms += tot_ns / c / 1e6 if c else 0.0
        calls = max(calls, c)
    rd = 2.0 * fetch * 1024
    wr = write * 1024
    out = {"kernel": bench_kernel, "kernel_match": sub, "launches_fetch_pass": nf, "launches_write_pass": nw,
           "fetch_bytes_per_launch": rd, "write_bytes_per_launch": wr, "traffic_bytes_per_launch": rd + wr,
           "rocprof_avg_launch_ms": avg_ms, "rocprof_calls": calls,
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count of wide streaming reads), WRITE_SIZE KiB x1024",
           "source": "tools/profile_round.sh: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) of "
                     "`python3 bench.py --no-cpu-baseline --no-gae-roofline`"}
    mfma = mfma_util(os.path.join(OUT, "pmcb", "mfma_counter_collection.csv"))
    if mfma:
        json.dump({"tag": tag, "workload": json.loads(line)["config"]["workload"],
                   "definition": "util = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / XCDs); "
                                 "SIMDs = 1024, XCDs = 8 (GRBM_GUI_ACTIVE sums the 8 XCDs); "
                                 "sclk_ghz = GRBM_GUI_ACTIVE / XCDs / the same dispatches' duration "
                                 "(End - Start timestamps of the counter pass)",
                   "kernels": mfma}, open(os.path.join(prof, f"{tag}_mfma.json"), "w"), indent=1)
        out["mfma_util_file"] = f"profiles/{tag}_mfma.json"
    out["tag"] = tag
    out["workload"] = json.loads(line)["config"]["workload"]   # bench.py only uses traffic of the same workload
    json.dump(out, open(os.path.join(prof, f"{tag}_traffic.json"), "w"), indent=1)
    # the file bench.py reads to fill roofline.traffic for this kernel
    json.dump(out, open(os.path.join(prof, "roofline_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
