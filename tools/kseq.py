#!/usr/bin/env python3
"""Instruction-class skeleton of one kernel's gfx950 code, for checking where a
schedule puts its global loads / stores, waits and barriers:
  python tools/kseq.py csrc/gemm.hip mangled_name_substring [--waits]   (in ppo-dash_amd/)
M mfma, L global/buffer load, S global/buffer store, D LDS-DMA load, r/W ds read/write,
w s_waitcnt with a vmcnt, | s_barrier; one line per basic block.  --waits lists the
vmcnt waits with their line in the kernel body; --mem prints every global / buffer
load, store and atomic, poll load, vmcnt wait, barrier, sleep and branch target with
its line (the order evidence for a hand-off protocol)."""
import re
import subprocess
import sys

src, pat = sys.argv[1], sys.argv[2]
asm = subprocess.run(["/opt/rocm/lib/llvm/bin/clang++", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                      "-fvisibility=hidden", "--cuda-device-only", "-S", "-x", "hip", src, "-o", "-"],
                     capture_output=True, text=True, check=True).stdout
m = re.search(r"^(_Z\S*" + re.escape(pat) + r"\S*):", asm, re.M)
if not m:
    sys.exit(f"no kernel matching {pat}")
body = asm[m.end():asm.find(".Lfunc_end", m.end())].split("\n")
print(m.group(1))
if "--mem" in sys.argv:
    for i, ln in enumerate(body):
        t = ln.strip()
        if (t.startswith(("s_barrier", "buffer_load", "buffer_store", "global_load", "global_store", "global_atomic",
                          "s_sleep", ".LBB")) or (t.startswith("s_waitcnt") and "vmcnt" in t)):
            print(f"{i:5d} {t.split(';')[0].rstrip()[:110]}")
    sys.exit(0)
out = []
for i, ln in enumerate(body):
    t = ln.strip().split(" ")[0]
    if t.startswith("v_mfma"):
        c = "M"
    elif (t.startswith("buffer_load") or t.startswith("global_load")) and " lds" in ln:
        c = "D"
    elif t.startswith("buffer_load") or t.startswith("global_load"):
        c = "L"
    elif t.startswith("buffer_store") or t.startswith("global_store"):
        c = "S"
    elif t == "s_barrier":
        c = "|"
    elif t.startswith("s_waitcnt") and "vmcnt" in ln:
        c = "w"
        if "--waits" in sys.argv:
            print(f"  {i}: {ln.strip()}")
    elif t.startswith("ds_write"):
        c = "W"
    elif t.startswith("ds_read"):
        c = "r"
    elif t.startswith(".LBB"):
        c = "\n" + t + " "
    else:
        continue
    out.append(c)
print("".join(out))
