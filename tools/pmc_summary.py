#!/usr/bin/env python3
"""Reduce the counter passes of tools/pmc_sq.sh to one JSON per workload: per counter the median
over the main-grid dispatches of the dominant kernel, plus the derived occupancy and wait shares.
    python tools/pmc_summary.py OUT.json KERNEL_SUBSTRING pass1.csv [pass2.csv ...]
SQ_WAVE_CYCLES and the SQ_WAIT_* / SQ_ACTIVE_* counters count quad-cycles (MI355X_MICROARCH.md);
GRBM_GUI_ACTIVE sums the 8 XCDs."""
import csv
import json
import statistics
import sys

out, kname, paths = sys.argv[1], sys.argv[2], sys.argv[3:]
vals = {}
for p in paths:
    rows = [r for r in csv.DictReader(open(p)) if kname in r["Kernel_Name"]]
    if not rows:
        continue
    big = max(int(r["Grid_Size"]) for r in rows)
    by = {}
    for r in rows:
        if int(r["Grid_Size"]) != big:
            continue
        by.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
        by[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, d in by.items():
        vals[c] = statistics.median(d.values())
res = {"kernel": kname, "counters_median_per_dispatch": vals}
cus = 256
if "SQ_WAVE_CYCLES" in vals and "GRBM_GUI_ACTIVE" in vals:
    cyc = vals["GRBM_GUI_ACTIVE"] / 8
    wc = vals["SQ_WAVE_CYCLES"]
    res["kernel_cycles_per_xcd"] = cyc
    res["avg_waves_resident_per_cu"] = round(4 * wc / (cus * cyc), 2)
    if "SQ_WAVES" in vals:
        res["wave_life_cycles"] = round(4 * wc / vals["SQ_WAVES"], 1)
    for c, k in (("SQ_WAIT_ANY", "share_wait_any"), ("SQ_WAIT_INST_ANY", "share_wait_inst_any"),
                 ("SQ_ACTIVE_INST_ANY", "share_active_inst_any")):
        if c in vals:
            res[k] = round(vals[c] / wc, 3)
if "GRBM_GUI_ACTIVE" in vals:
    cyc = vals["GRBM_GUI_ACTIVE"] / 8
    for c in ("TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum",
              "TA_ADDR_STALLED_BY_TD_CYCLES_sum", "TD_TD_BUSY_sum", "TD_TC_STALL_sum",
              "TCP_PENDING_STALL_CYCLES_sum"):
        if c in vals:  # per CU, as a share of the kernel's cycles
            res[c.replace("_sum", "") + "_share"] = round(vals[c] / cus / cyc, 3)
    vm = vals.get("SQ_INSTS_VMEM_RD", 0) + vals.get("SQ_INSTS_VMEM_WR", 0)
    if vm and "TA_TA_BUSY_sum" in vals:
        res["TA_busy_cycles_per_vmem_inst"] = round(vals["TA_TA_BUSY_sum"] / vm, 2)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters_median_per_dispatch"}))
