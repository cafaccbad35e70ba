#!/usr/bin/env python3
"""Counters of the headline transpose against the copies of the same bytes in one bench run
(r5: what separates them).  python tools/pmc_compare.py <session dir with p*/ passes>
Per kernel (median over its dispatches of each counter), derived per launch:
  queue depth  TCC_EA0_{RD,WR}REQ_LEVEL / GRBM_GUI_ACTIVE (requests outstanding to memory, summed
               over the 16 L2 channels of each XCD, averaged over the kernel)
  EA latency   LEVEL / REQ x kernel cycles ... (Little: outstanding / rate)
  stalls       credit stalls towards DRAM per kernel cycle
  TA->L2       TCP_TCC_{READ,WRITE}_REQ_LATENCY / requests (cycles per request)
  UTCL1        translation misses per request"""
import csv
import glob
import statistics
import sys

KERNELS = {"tile_kernel<double": "transpose (tile_kernel fp64 64x128)", "seg_copy_1(": "copy 1 vec/thread, 4 cols (kind 4)",
           "flat_copy_1k(": "flat copy 1 KiB/wave (kind 3)", "seg_copy(": "strided copy 4 vec/thread (kind 1)",
           "flat_copy(": "flat copy 16 KiB/WG (kind 2)"}


def main():
    d = sys.argv[1]
    vals = {}  # (kernel label, counter) -> [values per dispatch]
    dur = {}
    for f in glob.glob(f"{d}/p*/*counter_collection.csv"):
        per = {}
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            lab = next((v for k, v in KERNELS.items() if k in name), None)
            if lab is None:
                continue
            key = (lab, r["Counter_Name"], r["Dispatch_Id"])
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
            dur.setdefault(lab, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for (lab, c, _), v in per.items():
            vals.setdefault((lab, c), []).append(v)
    med = {k: statistics.median(v) for k, v in vals.items()}
    labs = [v for v in KERNELS.values() if any(k[0] == v for k in med)]
    counters = sorted({c for _, c in med})
    print("%-44s" % "counter (median per dispatch)" + "".join("%26s" % l[:24] for l in labs))
    for c in counters:
        print("%-44s" % c + "".join("%26.4g" % med.get((l, c), float("nan")) for l in labs))

    def ratio(l, a, b):
        x, y = med.get((l, a)), med.get((l, b))
        return x / y if x is not None and y else float("nan")
    print()
    derived = [("read queue (RDREQ_LEVEL/GUI_ACTIVE)", "TCC_EA0_RDREQ_LEVEL_sum", "GRBM_GUI_ACTIVE"),
               ("write queue (WRREQ_LEVEL/GUI_ACTIVE)", "TCC_EA0_WRREQ_LEVEL_sum", "GRBM_GUI_ACTIVE"),
               ("read level per read request", "TCC_EA0_RDREQ_LEVEL_sum", "TCC_EA0_RDREQ_sum"),
               ("write level per write request", "TCC_EA0_WRREQ_LEVEL_sum", "TCC_EA0_WRREQ_sum"),
               ("DRAM read credit stall / GUI_ACTIVE", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "GRBM_GUI_ACTIVE"),
               ("DRAM write credit stall / GUI_ACTIVE", "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "GRBM_GUI_ACTIVE"),
               ("EA write stall / GUI_ACTIVE", "TCC_EA0_WRREQ_STALL_sum", "GRBM_GUI_ACTIVE"),
               ("tag stall / GUI_ACTIVE", "TCC_TAG_STALL_sum", "GRBM_GUI_ACTIVE"),
               ("TA->L2 read latency / request", "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum"),
               ("TA->L2 write latency / request", "TCP_TCC_WRITE_REQ_LATENCY_sum", "TCP_TCC_WRITE_REQ_sum"),
               ("UTCL1 misses / UTCL1 requests", "TCP_UTCL1_TRANSLATION_MISS_sum", "TCP_UTCL1_REQUEST_sum"),
               ("UTCL1 inflight-max stall / GUI_ACTIVE", "TCP_UTCL1_STALL_INFLIGHT_MAX_sum", "GRBM_GUI_ACTIVE"),
               ("TCP pending stall / GUI_ACTIVE", "TCP_PENDING_STALL_CYCLES_sum", "GRBM_GUI_ACTIVE"),
               ("waves resident (SQ_LEVEL_WAVES/SQ_BUSY)", "SQ_LEVEL_WAVES", "SQ_BUSY_CYCLES"),
               ("wait-any share (SQ_WAIT_ANY/SQ_WAVE_CYCLES)", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES")]
    for name, a, b in derived:
        print("%-44s" % name + "".join("%26.4g" % ratio(l, a, b) for l in labs))
    print("%-44s" % "kernel ms (PMC runs)" + "".join("%26.4g" % (statistics.median(dur[l]) / 1e6) for l in labs))


if __name__ == "__main__":
    main()
