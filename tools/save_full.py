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
import time

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


def counter(base, kind, kern):
    """median per dispatch of the largest-grid `kern` launch in one --pmc pass, KiB"""
    files = glob.glob(os.path.join(base, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != kind or kern not in r["Kernel_Name"]:
                continue
            g = int(r["Grid_Size"])
            vals.setdefault(g, []).append(float(r["Counter_Value"]))
    if not vals:
        return None, None
    g = max(vals)
    return statistics.median(vals[g]), {"grid": g, "dispatches": len(vals[g])}


def save_pmc(fetch_dir, write_dir, log, kern, name, read_share):
    """one workload's HBM traffic per launch from its FETCH_SIZE and WRITE_SIZE passes;
    read_share: the algorithmic reads' share of the algorithmic bytes"""
    # several kernels of one phase (cfg 5: the destination-block groups and the wavefront
    # pieces): each kernel's largest-grid median, summed
    kerns = kern if isinstance(kern, tuple) else (kern,)
    fk = wk = 0.0
    fi, wi = {}, {}
    for k in kerns:
        f1, i1 = counter(fetch_dir, "FETCH_SIZE", k)
        w1, j1 = counter(write_dir, "WRITE_SIZE", k)
        if f1 is None or w1 is None:
            continue
        fk, wk = fk + f1, wk + w1
        fi[k], wi[k] = i1, j1
    if not fi:
        fk = wk = None
    kern = " + ".join(kerns)
    d = line(log) if os.path.exists(log) else None
    if fk is None or wk is None or not d:
        return
    alg = d["roofline"]["bytes_per_launch"]
    out = {"FETCH_SIZE_KiB": fk, "WRITE_SIZE_KiB": wk, "fetch": fi, "write": wi, "kernel": kern,
           "hbm_bytes_per_launch_corrected": int((2 * fk + wk) * 1024),
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving)",
           "bytes_per_launch_alg": alg, "workload": d["config"]["workload"],
           "collected": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(os.path.getmtime(log)))}
    out["ratio_to_algorithmic"] = round(out["hbm_bytes_per_launch_corrected"] / alg, 4)
    out["reads_to_algorithmic"] = round(2 * fk * 1024 / (alg * read_share), 4)
    out["writes_to_algorithmic"] = round(wk * 1024 / (alg * (1 - read_share)), 4)
    json.dump(out, open(os.path.join(dst, name), "w"), indent=1)
    print(name, {k: v for k, v in out.items() if k not in ("fetch", "write", "correction", "workload")})


# the cfg 2 launch (tools/gpu_full.sh); cfg 5 'N' / 'T' when tools/c5_pmc.sh ran as <tag>_c5pmc
save_pmc(os.path.join(src, "pmc_FETCH_SIZE"), os.path.join(src, "pmc_WRITE_SIZE"),
         os.path.join(src, "pmc_FETCH_SIZE.log"), "tile_kernel<double", "pmc_tile_kernel.json", 0.5)
c5 = src + "_c5pmc"
for op, share in (("N", 0.5), ("T", 2 / 3)):
    save_pmc(os.path.join(c5, f"pmc_{op}_FETCH_SIZE"), os.path.join(c5, f"pmc_{op}_WRITE_SIZE"),
             os.path.join(c5, f"pmc_{op}_FETCH_SIZE.log"), ("cblock_kernel<float", "tiny_kernel<float"),
             f"pmc_cfg5_{op}.json", share)
    st = os.path.join(c5, f"prof_{op}", "trace_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(dst, f"c5{op}_trace_kernel_stats.csv"))
# cfg 4 / cfg 3 single-GPU slices when tools/c34_prof.sh ran as <tag>_c34
c34 = src + "_c34"
for n, kern, share in (("cfg4", "tile_kernel<costa::engine::(anonymous namespace)::cpx<double>", 2 / 3),
                       ("cfg3", "tile_kernel<double", 0.5)):
    save_pmc(os.path.join(c34, f"pmc_{n}_FETCH_SIZE"), os.path.join(c34, f"pmc_{n}_WRITE_SIZE"),
             os.path.join(c34, f"pmc_{n}_FETCH_SIZE.log"), kern, f"pmc_{n}.json", share)
    st = os.path.join(c34, f"prof_{n}", "trace_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(dst, f"{n}_trace_kernel_stats.csv"))
    lg = os.path.join(c34, f"prof_{n}.log")
    if os.path.exists(lg) and line(lg):
        json.dump(line(lg), open(os.path.join(dst, f"{n}.json"), "w"))
for name in ("bench.json", "c5N.json", "c5T.json", "extra.json", "cfg4.json", "cfg3.json"):
    d = line(os.path.join(dst, name))
    if d:
        print(name, d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["avg_launch_ms"],
              d["verified"])
print("saved", dst)
