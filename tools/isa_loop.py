#!/usr/bin/env python3
"""Instruction mix of a kernel's hottest loop (container-side, no GPU).

  python tools/isa_loop.py FILE.s 'igemm_x9_kernel.*DenseReluFwd.*XP128' [--all]

FILE.s comes from `hipcc --offload-arch=gfx950 --cuda-device-only -O3 -S csrc/gemm.hip`.
For each function whose (mangled) name matches the regex, the loops (a label that a
later s_cbranch / s_branch jumps back to) are listed with their instruction counts by
class; without --all only the loop holding the most MFMAs is shown.
"""
import re
import sys
from collections import Counter


def functions(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^([A-Za-z_][\w.$]*):\s*(;.*)?$", line)
        if m and not m.group(1).startswith(".") and line.startswith(m.group(1)):
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur:
            if line.startswith("\t.size") or line.startswith("\t.end_amdhsa_kernel"):
                yield cur, body
                cur, body = None, []
            else:
                body.append(line.rstrip("\n"))
    if cur:
        yield cur, body


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith(("global_load", "buffer_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store")):
        return "vmem_store"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "lds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "lds_write"
    if op.startswith("s_waitcnt") or op in ("s_barrier", "s_nop", "s_setprio"):
        return "sync"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def loops(body):
    labels = {}
    insts = []
    for line in body:
        s = line.strip()
        m = re.match(r"^(\.LBB[\w_]+):", s)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        insts.append((op, s))
    out = []
    for i, (op, s) in enumerate(insts):
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                seg = insts[labels[tgt]:i + 1]
                out.append((tgt, seg))
    return out


def main():
    path, rx = sys.argv[1], re.compile(sys.argv[2])
    show_all = "--all" in sys.argv
    for name, body in functions(path):
        if not rx.search(name):
            continue
        ls = loops(body)
        if not ls:
            continue
        if not show_all:
            ls = [max(ls, key=lambda t: sum("mfma" in o for o, _ in t[1]))]
        print(name)
        for tgt, seg in ls:
            cls = Counter(classify(o) for o, _ in seg)
            ops = Counter(o for o, _ in seg)
            print(f"  loop {tgt}: {len(seg)} insts  " + "  ".join(f"{k}={v}" for k, v in sorted(cls.items())))
            print("    top: " + "  ".join(f"{k}={v}" for k, v in ops.most_common(14)))


if __name__ == "__main__":
    main()
