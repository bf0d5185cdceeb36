#!/usr/bin/env python3
"""Average PMC counters per launch of kernels matching a substring, from the
tools/pmc_one.sh output (gpurun_out/pmc1/p*_counter_collection.csv).
  python tools/pmc_parse.py conv2_dgrad_x9 [dir]"""
import collections
import csv
import glob
import os
import sys

pat = sys.argv[1]
d = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/pmc1"
for f in sorted(glob.glob(os.path.join(d, "p*_counter_collection.csv"))):
    agg, n = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
    print(os.path.basename(f), {k: f"{v / n[k]:.3e}" for k, v in sorted(agg.items())})
