#!/usr/bin/env python3
"""Copy one tools/gpu_full.sh session (gpurun_out/<tag>/) into profiles/<tag>/:
  bench / cfg 5 / extra JSON lines, the -m gpu and smoke logs (tails), the rocprofv3 kernel
  statistics of the bench, a per-dispatch summary (kernel_dispatches.json), and the HBM traffic
  per launch from the FETCH_SIZE / WRITE_SIZE passes, corrected as MI355X_MICROARCH.md prescribes
  for gfx950 (FETCH_SIZE counts half of a wide streaming read: doubled; KiB -> bytes).
bench.py's measured_traffic() picks pmc_*.json by bytes_per_launch_alg.
    python tools/save_full.py r3t"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

tag = sys.argv[1]
src = os.path.join("gpurun_out", tag)
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)

for name in ("bench.json", "c5N.json", "c5T.json", "extra.json", "smoke.log"):
    p = os.path.join(src, name)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, name))
for name in ("pytest_gpu.log",):
    p = os.path.join(src, name)
    if os.path.exists(p):
        lines = open(p).read().splitlines()
        open(os.path.join(dst, name.replace(".log", "_tail.txt")), "w").write("\n".join(lines[-5:]) + "\n")
p = os.path.join(src, "prof", "trace_kernel_stats.csv")
if os.path.exists(p):
    shutil.copy(p, os.path.join(dst, "trace_kernel_stats.csv"))


def line(path):
    try:
        return json.loads([l for l in open(path) if l.startswith("{")][-1])
    except Exception:
        return None


# per kernel and grid: dispatches, mean / median duration (the stats CSV mixes every grid size)
tr = os.path.join(src, "prof", "trace_kernel_trace.csv")
if os.path.exists(tr):
    by = {}
    for r in csv.DictReader(open(tr)):
        if "costa" not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
        by.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = [{"kernel": k[0], "grid": k[1], "workgroup": k[2], "dispatches": len(v),
            "mean_ns": round(statistics.mean(v), 1), "median_ns": statistics.median(v)}
           for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))]
    json.dump(out, open(os.path.join(dst, "kernel_dispatches.json"), "w"), indent=1)


def counter(kind):
    """median per dispatch of the largest-grid tile_kernel<double> (the cfg 2 launch), KiB"""
    files = glob.glob(os.path.join(src, f"pmc_{kind}", "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != kind or "tile_kernel<double" not in r["Kernel_Name"]:
                continue
            g = int(r["Grid_Size"])
            vals.setdefault(g, []).append(float(r["Counter_Value"]))
    if not vals:
        return None, None
    g = max(vals)
    return statistics.median(vals[g]), {"grid": g, "dispatches": len(vals[g])}


fk, fi = counter("FETCH_SIZE")
wk, wi = counter("WRITE_SIZE")
d = line(os.path.join(src, "pmc_FETCH_SIZE.log"))
if fk is not None and wk is not None and d:
    out = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk, "fetch": fi, "write": wi,
           "hbm_bytes_per_launch_corrected": int((2 * fk + wk) * 1024),
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)",
           "bytes_per_launch_alg": d["roofline"]["bytes_per_launch"],
           "workload": d["config"]["workload"]}
    out["ratio_to_algorithmic"] = round(out["hbm_bytes_per_launch_corrected"] / out["bytes_per_launch_alg"], 4)
    json.dump(out, open(os.path.join(dst, "pmc_tile_kernel.json"), "w"), indent=1)
    print("pmc", {k: v for k, v in out.items() if k not in ("fetch", "write")})
for name in ("bench.json", "c5N.json", "c5T.json", "extra.json"):
    d = line(os.path.join(dst, name))
    if d:
        print(name, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"],
              d["verified"])
print("saved", dst)
