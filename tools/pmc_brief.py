#!/usr/bin/env python3
"""Per-kernel median of one rocprofv3 --pmc pass (counter_collection.csv under <dir>), for the
costa kernels of the largest grid: python tools/pmc_brief.py <dir> [<alg bytes per launch>]
FETCH_SIZE is doubled (gfx950 correction, MI355X_MICROARCH.md; exact for dword, 16-byte and
partial-line loads: profiles/r6c/, tools/pmc_bytes.py), values in KiB -> bytes."""
import csv
import glob
import statistics
import sys

d = sys.argv[1]
alg = float(sys.argv[2]) if len(sys.argv) > 2 else None
files = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
by = {}
for f in files:
    for r in csv.DictReader(open(f)):
        if "costa" not in r["Kernel_Name"]:
            continue
        key = (r["Counter_Name"], r["Kernel_Name"].split("(")[0][-60:], int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0))
        by.setdefault(key, {}).setdefault(r.get("Dispatch_Id", r.get("Correlation_Id")), 0.0)
        by[key][r.get("Dispatch_Id", r.get("Correlation_Id"))] += float(r["Counter_Value"])
for (c, k, g), v in sorted(by.items(), key=lambda kv: -kv[0][2]):
    med = statistics.median(v.values())
    b = med * 1024 * (2 if c == "FETCH_SIZE" else 1)
    extra = f" = {b / alg:.3f} x alg" if alg else ""
    print(f"{c:12s} grid {g:>10d} n={len(v):3d} median {b / 1e6:10.2f} MB{extra}  {k}")
