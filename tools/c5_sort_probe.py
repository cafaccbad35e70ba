"""Tuning probe (not product): per-phase kernel time of BASELINE cfg 5 (bench.py's workload)
under the wavefront sort modes (COSTA_TUNING=1 COSTA_TINY_SORT, engine.cpp wave_knobs::sort).  With
COSTA_LOOPBACK=1 every tile goes through PACK -> RCCL self send/recv -> UNPACK, so the pack and
unpack lists of a multi-rank run are timed on one GPU.
    COSTA_TINY_SORT=5 COSTA_LOOPBACK=1 python tools/c5_sort_probe.py N [steps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import costa_amd as costa  # noqa: E402


def main():
    op = sys.argv[1] if len(sys.argv) > 1 else "N"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    costa.lib()
    comm = costa.Comm.self(0)
    LA, LC, A, C, op, al, be, wl, masks, _ca = bench.cfg5_workload(costa, torch, 0, 1, op)
    for _ in range(3):
        costa.transform_async(LA, LC, comm, op, al, be)
    costa.synchronize(comm)
    costa.set_profiling(True)
    costa.get_stats(reset=True)
    for _ in range(steps):
        costa.transform_async(LA, LC, comm, op, al, be)
    costa.synchronize(comm)
    st = costa.get_stats(reset=True)
    parts = []
    for k in ("pack", "local", "unpack"):
        if st[k + "_launches"]:
            ms = st[k + "_ms"] / steps
            parts.append(f"{k} {ms:.4f} ms {st[k + '_bytes'] / steps / (ms * 1e-3) / 1e9:7.1f} GB/s")
    print(f"sort={os.environ.get('COSTA_TINY_SORT', 'default')} loopback={os.environ.get('COSTA_LOOPBACK', '0')} "
          f"op {op}: " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
