#!/usr/bin/env python3
"""Register / scratch / LDS use of the gfx950 kernels of one source file, from the
code-object metadata of a device-only assembly build:
  python tools/kres.py csrc/gemm.hip [name_substring ...]   (run in ppo-dash_amd/)"""
import re
import subprocess
import sys

src, pats = sys.argv[1], sys.argv[2:]
asm = subprocess.run(["/opt/rocm/lib/llvm/bin/clang++", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                      "-fvisibility=hidden", "--cuda-device-only", "-S", "-x", "hip", src, "-o", "-"],
                     capture_output=True, text=True, check=True).stdout
meta = asm[asm.index("amdhsa.kernels:"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    f = dict(re.findall(r"^\s*\.(\w+):\s+(\S+)", blk, re.M))
    name = f.get("name", "?")
    if pats and not any(p in name for p in pats):
        continue
    print(f"{name[:90]:90s} vgpr {f.get('vgpr_count')} agpr {f.get('agpr_count')} "
          f"scratch {f.get('private_segment_fixed_size')} lds {f.get('group_segment_fixed_size')} "
          f"spill {f.get('vgpr_spill_count')}")
