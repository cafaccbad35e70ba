#!/usr/bin/env python3
"""Counters of the headline transpose split by placement mode (r5): the dispatches of
tools/pairs_probe.py under rocprofv3 --pmc fall into two duration clusters (fast / slow physical
placement of the pair); per counter the median of each cluster, and their ratio.
    python tools/pmc_modes.py <session dir with p*/ passes> [split ms]"""
import csv
import glob
import statistics
import sys


def main():
    d = sys.argv[1]
    split = float(sys.argv[2]) if len(sys.argv) > 2 else 0.68
    rows = []
    for f in sorted(glob.glob(f"{d}/p*/*counter_collection.csv")):
        per, dur = {}, {}
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            lab = "tile" if "tile_kernel<double" in name else "copy" if "seg_copy_1(" in name else None
            if lab is None:
                continue
            k = (lab, r["Dispatch_Id"])
            per.setdefault(r["Counter_Name"], {}).setdefault(k, 0.0)
            per[r["Counter_Name"]][k] += float(r["Counter_Value"])
            dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        for c, v in per.items():
            for lab in ("tile", "copy"):
                fast = [x for k, x in v.items() if k[0] == lab and dur[k] < split + (0 if lab == "tile" else -0.04)]
                slow = [x for k, x in v.items() if k[0] == lab and dur[k] >= split + (0 if lab == "tile" else -0.04)]
                if fast and slow:
                    mf, ms = statistics.median(fast), statistics.median(slow)
                    rows.append((lab, c, len(fast), mf, len(slow), ms, ms / mf if mf else float("nan")))
        tiles = sorted(v for k, v in dur.items() if k[0] == "tile")
        if tiles:
            print(f"{f.split('/')[-2]}: tile dispatches {len(tiles)}, ms {tiles[0]:.4f} .. {tiles[-1]:.4f}")
    print(f"{'kernel':5s} {'counter':42s} {'fast n':>6s} {'fast median':>14s} {'slow n':>6s} {'slow median':>14s} {'slow/fast':>9s}")
    for lab, c, nf, mf, ns, ms, q in rows:
        print(f"{lab:5s} {c:42s} {nf:6d} {mf:14.5g} {ns:6d} {ms:14.5g} {q:9.3f}")


if __name__ == "__main__":
    main()
