#!/usr/bin/env python3
"""Per-launch SQ counters and derived wave-cycle shares of kernels from the
tools/pmc_sq.sh passes (gpurun_out/pmc1/p*_counter_collection.csv), as in
profiles/r03_v2_sq.json:
  python tools/sq_summary.py TAG name_substring[,name_substring...] [dir]
Shares are of SQ_WAVE_CYCLES: waiting = SQ_WAIT_ANY (s_waitcnt / barrier),
issue-stalled = SQ_WAIT_INST_ANY, issuing = SQ_ACTIVE_INST_ANY; MFMA utilisation =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128) (GRBM summed over the 8 XCDs,
32 CUs x 4 SIMDs per XCD)."""
import collections
import csv
import glob
import json
import os
import sys

tag, pats = sys.argv[1], sys.argv[2].split(",")
d = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/pmc1"
out = {"tag": tag, "source": "tools/pmc_sq.sh (rocprofv3 --pmc passes of tools/kbench.py at the c3 minibatch)",
       "kernels": {}}
for pat in pats:
    agg, n = collections.defaultdict(float), collections.Counter()
    for f in sorted(glob.glob(os.path.join(d, "**", "p*_counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
    pl = {k: v / n[k] for k, v in agg.items()}
    if not pl:
        continue
    e = {"per_launch": {k: round(v) for k, v in sorted(pl.items())}}
    wc = pl.get("SQ_WAVE_CYCLES")
    if wc:
        e["wave_cycle_shares"] = {"waiting (s_waitcnt / barrier)": round(pl.get("SQ_WAIT_ANY", 0) / wc, 3),
                                  "issue-stalled": round(pl.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                                  "issuing": round(pl.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3),
                                  "LDS issue stall": round(pl.get("SQ_WAIT_INST_LDS", 0) / wc, 3)}
    m = pl.get("SQ_INSTS_MFMA")
    if m:
        for k, name in (("SQ_INSTS_VALU", "valu_per_mfma"), ("SQ_INSTS_LDS", "lds_per_mfma"),
                        ("SQ_INSTS_SALU", "salu_per_mfma")):
            if k in pl:
                e[name] = round(pl[k] / m, 2)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in pl and "GRBM_GUI_ACTIVE" in pl:
        e["mfma_util"] = round(pl["SQ_VALU_MFMA_BUSY_CYCLES"] / (pl["GRBM_GUI_ACTIVE"] * 128), 3)
    if "SQ_LDS_BANK_CONFLICT" in pl and pl.get("SQ_LDS_IDX_ACTIVE"):
        e["lds_bank_conflict_share"] = round(pl["SQ_LDS_BANK_CONFLICT"] / pl["SQ_LDS_IDX_ACTIVE"], 3)
    out["kernels"][pat] = e
print(json.dumps(out, indent=1))
