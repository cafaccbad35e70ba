#!/usr/bin/env python3
"""Copy one gpu_check.sh session's summaries from gpurun_out/<tag>/ into profiles/<tag>/ and
derive the HBM traffic per launch phase from the PMC passes, corrected as MI355X_MICROARCH.md
prescribes for gfx950 (FETCH_SIZE reports half of a wide streaming read: double it;
WRITE_SIZE exact for 16-B stores; both in KiB).

A bench step's phase may run several kernels (tile_kernel for large ops, tiny_kernel for the
wavefront path): for each kernel name of the workload's element type the dispatches of its main
grid are taken, the median per kernel is summed.  One json per workload:
  pmc_tile_kernel.json  (default bench, BASELINE cfg 2)
  pmc_cfg5_N.json / pmc_cfg5_T.json
bench.py's measured_traffic() picks the file whose bytes_per_launch_alg equals its own.
The x2 FETCH correction is exact for every access width the kernels use (r6, profiles/r6c/:
TCC_EA0_RDREQ_128B / _64B / _32B show that gfx950's L2 reads memory in whole 128-byte lines for
dword, 16-byte and partial-line loads alike, FETCH_SIZE tallying each at 64 B;
tools/pmc_bytes.py computes the bytes from those counters directly)."""
import csv
import json
import os
import shutil
import statistics
import sys

tag = sys.argv[1]
src = os.path.join("gpurun_out", tag)
dst = os.path.join("profiles", tag)
os.makedirs(dst, exist_ok=True)
for rel in ["prof/trace_kernel_stats.csv", "bench.log", "pytest_gpu.log", "smoke.log", "nproc.txt",
            "gpu.txt", "c5N_prof/trace_kernel_stats.csv", "c5T_prof/trace_kernel_stats.csv",
            "c5N_bench.log", "c5T_bench.log", "c5_knobs.log"]:
    p = os.path.join(src, rel)
    if os.path.exists(p):
        name = rel.replace("/", "_") if rel.startswith("c5") else os.path.basename(rel)
        shutil.copy(p, os.path.join(dst, name))


def dispatch_summary():
    """per kernel and grid size: dispatch count, mean and median duration (ns), from each
    kernel trace of the session (a kernel's rocprofv3 stats average mixes every launch size of
    it; the workload's own launches are the largest grid)"""
    out = {}
    for sub in ("prof", "c5N_prof", "c5T_prof"):
        p = os.path.join(src, sub, "trace_kernel_trace.csv")
        if not os.path.exists(p):
            continue
        by = {}
        for r in csv.DictReader(open(p)):
            if "costa" not in r["Kernel_Name"]:
                continue
            k = (r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
            by.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        out[sub] = [{"kernel": k[0], "grid": k[1], "workgroup": k[2], "dispatches": len(v),
                     "mean_ns": round(statistics.mean(v), 1), "median_ns": statistics.median(v)}
                    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))]
    if out:
        json.dump(out, open(os.path.join(dst, "kernel_dispatches.json"), "w"), indent=1)


def bench_line(path):
    try:
        return json.loads([l for l in open(path) if l.startswith("{")][-1])
    except Exception:
        return None


def phase_kib(csv_path, counter, dtype):
    """sum over the phase's kernels (tile_kernel / tiny_kernel of `dtype`) of the median
    counter value of each kernel's main-grid dispatches"""
    rows = [r for r in csv.DictReader(open(csv_path)) if r["Counter_Name"] == counter]
    total, per = 0.0, {}
    for kname in ("tile_kernel", "tiny_kernel"):
        rs = [r for r in rows if f"{kname}<{dtype}" in r["Kernel_Name"]]
        if not rs:
            continue
        big = max(int(r["Grid_Size"]) for r in rs)
        vals = [float(r["Counter_Value"]) for r in rs if int(r["Grid_Size"]) == big]
        per[kname] = {"grid": big, "dispatches": len(vals), "median_KiB": statistics.median(vals)}
        total += statistics.median(vals)
    return total, per


def derive(prefix, dtype, out_name):
    f = os.path.join(src, f"{prefix}pmc_fetch/fetch_counter_collection.csv")
    w = os.path.join(src, f"{prefix}pmc_write/write_counter_collection.csv")
    if not (os.path.exists(f) and os.path.exists(w)):
        return
    fk, fper = phase_kib(f, "FETCH_SIZE", dtype)
    wk, wper = phase_kib(w, "WRITE_SIZE", dtype)
    out = {"FETCH_SIZE_KiB_per_phase": fk, "WRITE_SIZE_KiB_per_phase": wk,
           "kernels_fetch": fper, "kernels_write": wper,
           "hbm_bytes_per_launch_corrected": int((2 * fk + wk) * 1024),
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE halving; "
                         "exact for dword, 16-byte and partial-line loads: every memory read is a 128-byte "
                         "request, profiles/r6c/)"}
    d = bench_line(os.path.join(src, f"{prefix}pmc_fetch.log"))
    if d:
        out["bytes_per_launch_alg"] = d["roofline"]["bytes_per_launch"]
        out["workload"] = d["config"]["workload"]
        out["ratio_to_algorithmic"] = round(out["hbm_bytes_per_launch_corrected"] /
                                            out["bytes_per_launch_alg"], 4)
    json.dump(out, open(os.path.join(dst, out_name), "w"), indent=1)
    print(out_name, json.dumps({k: v for k, v in out.items() if not k.startswith("kernels")}))


dispatch_summary()
derive("", "double", "pmc_tile_kernel.json")
derive("c5N_", "float", "pmc_cfg5_N.json")
derive("c5T_", "float", "pmc_cfg5_T.json")
print("saved", dst)
