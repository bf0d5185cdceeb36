#!/bin/bash
# batch-1 eval act: timings and a kernel trace of the replay path
set -u
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
timeout -k 10 200 python tools/eval_probe.py || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/evalprof3 -o run -- python3 tools/eval_probe.py > gpurun_out/evalprof3.log 2>&1 || { tail -5 gpurun_out/evalprof3.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/evalprof3/**/run_kernel_trace.csv", recursive=True) or glob.glob("gpurun_out/evalprof3/run_kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 12 dispatches belong to the replay loop's final acts
tail = rows[-24:]
t0 = int(tail[0]["Start_Timestamp"])
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:6.1f} us  {r['Kernel_Name'][:90]}")
PY
