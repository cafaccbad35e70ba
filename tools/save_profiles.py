#!/usr/bin/env python3
"""Copy one gpu_check.sh session's summaries from gpurun_out/<tag>/ into profiles/<tag>/ and
derive the HBM traffic per launch of the tile kernel from the PMC passes, corrected as
MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE reports half of a wide streaming read:
double it; WRITE_SIZE exact for 16-B stores; both in KiB)."""
import csv
import json
import os
import shutil
import sys

tag = sys.argv[1]
src = os.path.join("gpurun_out", tag)
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)
for rel in ["prof/trace_kernel_stats.csv", "bench.log", "pytest_gpu.log", "smoke.log", "nproc.txt",
            "gpu.txt"]:
    p = os.path.join(src, rel)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, os.path.basename(rel)))
out = {}
for f, c in [("pmc_fetch/fetch_counter_collection.csv", "FETCH_SIZE"),
             ("pmc_write/write_counter_collection.csv", "WRITE_SIZE")]:
    p = os.path.join(src, f)
    if not os.path.exists(p):
        continue
    rows = [r for r in csv.DictReader(open(p))
            if "tile_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c]
    big = max(int(r["Grid_Size"]) for r in rows)  # the bench's dominant launch
    vals = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == big]
    out[c + "_KiB_per_launch"] = vals
if out:
    f = sorted(out.get("FETCH_SIZE_KiB_per_launch", [0]))
    w = sorted(out.get("WRITE_SIZE_KiB_per_launch", [0]))
    fm, wm = f[len(f) // 2], w[len(w) // 2]
    out["hbm_bytes_per_launch_corrected"] = int((2 * fm + wm) * 1024)
    try:
        line = [l for l in open(os.path.join(src, "bench.log")) if l.startswith("{")][-1]
        out["bytes_per_launch_alg"] = json.loads(line)["roofline"]["bytes_per_launch"]
    except Exception:
        pass
    out["correction"] = "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)"
    json.dump(out, open(os.path.join(dst, "pmc_tile_kernel.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if not k.endswith("launch")}))
print("saved", dst)
