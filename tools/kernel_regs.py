#!/usr/bin/env python3
"""VGPR / SGPR / scratch / LDS of every costa kernel in libcosta_amd.so (gfx950 code object
metadata), one line each: python tools/kernel_regs.py [lib] > before.txt"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "costa_amd", "lib", "libcosta_amd.so")
with tempfile.TemporaryDirectory() as td:
    shutil.copy(lib, os.path.join(td, "lib.so"))
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", "lib.so"], check=True, capture_output=True, cwd=td)
    for o in sorted(os.listdir(td)):
        if "gfx950" not in o:
            continue
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(td, o)], check=True,
                               capture_output=True, text=True).stdout
        rows = []
        for block in re.split(r"\n\s+- \.", notes):
            g = lambda k: (re.search(rf"\.{k}:\s+(\S+)", block) or [None, "?"])[1]
            name = g("name")
            if "costa" not in name:
                continue
            dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            dm = dm.replace("costa::engine::(anonymous namespace)::", "").split("(costa_tile_op_t")[0]
            rows.append(f"v{g('vgpr_count'):>4} s{g('sgpr_count'):>4} scr{g('private_segment_fixed_size'):>4} {dm}")
        print("\n".join(sorted(rows, key=lambda r: r.split(None, 3)[3])))
