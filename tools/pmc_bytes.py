#!/usr/bin/env python3
"""HBM read bytes from the L2's memory-side request counters by request size, per kernel (median
over its dispatches of the largest grid), with no correction factor:
    bytes = 128 x TCC_EA0_RDREQ_128B + 64 x TCC_EA0_RDREQ_64B + 32 x TCC_EA0_RDREQ_32B
FETCH_SIZE tallies every request at 64 B on gfx950: x2 is exact for streams of whole 128-byte
lines only (profiles/r6a: dword or 16-byte lanes alike); for partial lines the factor depends on
the pattern.  One rocprofv3 --pmc pass holds the four TCC counters:
    rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum ...
    python tools/pmc_bytes.py <pmc dir> [<algorithmic read bytes per launch>] [--all]
(--all: every kernel of the pass, not only the costa ones)"""
import csv
import glob
import statistics
import sys

SIZES = {"TCC_EA0_RDREQ_128B_sum": 128, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_32B_sum": 32}


def per_kernel(d, every=False):
    """-> {kernel name: {counter: median per dispatch}} for the largest grid of each kernel"""
    rows = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            if not every and "costa" not in name:
                continue
            g = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
            did = r.get("Dispatch_Id", r.get("Correlation_Id"))
            rows.setdefault(name, {}).setdefault(g, {}).setdefault(r["Counter_Name"], {}).setdefault(did, 0.0)
            rows[name][g][r["Counter_Name"]][did] += float(r["Counter_Value"])
    out = {}
    for name, grids in rows.items():
        g = max(grids)
        out[name] = {"grid": g, **{c: statistics.median(v.values()) for c, v in grids[g].items()}}
    return out


def main():
    d = sys.argv[1]
    alg = float(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    for name, c in sorted(per_kernel(d, "--all" in sys.argv).items(), key=lambda kv: -kv[1]["grid"]):
        if "TCC_EA0_RDREQ_128B_sum" not in c:
            continue
        b = sum(c.get(k, 0.0) * s for k, s in SIZES.items())
        n = sum(c.get(k, 0.0) for k in SIZES)
        tot = c.get("TCC_EA0_RDREQ_sum", float("nan"))
        extra = f" = {b / alg:.3f} x alg reads" if alg else ""
        print(f"{name[-70:]:70s} grid {c['grid']:>9d}: reads {b / 1e6:10.2f} MB{extra}  "
              f"(128B {c.get('TCC_EA0_RDREQ_128B_sum', 0):.0f}, 64B {c.get('TCC_EA0_RDREQ_64B_sum', 0):.0f}, "
              f"32B {c.get('TCC_EA0_RDREQ_32B_sum', 0):.0f}; sized {n:.0f} of {tot:.0f} requests; "
              f"FETCH_SIZE-style 64 B x all {64 * tot / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()
