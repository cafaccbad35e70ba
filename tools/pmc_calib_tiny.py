#!/usr/bin/env python3
"""Calibration (not product) of FETCH_SIZE / WRITE_SIZE for the wavefront path's 4-byte accesses.

MI355X_MICROARCH.md calibrates the gfx950 counters for 16-byte-per-lane streams only.  Here the
wavefront kernel (tiny_kernel<float>) runs on a geometry whose true HBM bytes are known: the cfg 5
generator with every block edge a multiple of 32 fp32 elements, so every tile column run starts
and ends on a 128-byte line on both sides and no line is shared between tiles.  The bytes moved
per launch are then exactly the algorithmic ones (A read, C written, C read when beta != 0; the
1 GiB buffers are far beyond the 256 MiB Infinity Cache).  Run one counter per rocprofv3 pass:
    rocprofv3 --pmc FETCH_SIZE -- python3 tools/pmc_calib_tiny.py N|T
The script prints the launch's algorithmic read / write bytes, which tools/save_profiles.py
divides by the counters to obtain the factors it applies to cfg 5."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import costa_amd as costa  # noqa: E402

N = 16384
Q = 32  # edge multiple: 32 fp32 = one 128-byte line


def splits(seed, lo, hi):
    r = np.random.default_rng(seed)
    s = [0]
    while s[-1] < N:
        e = int(r.integers(lo, hi + 1))
        e = max(Q, (e + Q // 2) // Q * Q)
        s.append(min(N, s[-1] + e))
    return s


def layout(rs, cs, buf):
    blocks, off = [], 0
    for i in range(len(rs) - 1):
        for j in range(len(cs) - 1):
            rows, cols = rs[i + 1] - rs[i], cs[j + 1] - cs[j]
            blocks.append((buf.data_ptr() + 4 * off, rows, i, j))
            off += (rows * cols + 63) // 64 * 64  # 256-byte aligned block starts
    own = np.zeros((len(rs) - 1, len(cs) - 1), np.int64)
    return costa.custom_layout(len(rs) - 1, len(cs) - 1, rs, cs, own, blocks, "C", costa.FLOAT)


op = sys.argv[1] if len(sys.argv) > 1 else "N"
al, be = (1.0, 0.0) if op == "N" else (-0.5, 2.0)
ars, acs = splits(0xC5A1, 8, 96), splits(0xC5A2, 8, 96)
crs, ccs = splits(0xC5A3, 16, 160), splits(0xC5A4, 16, 160)
A = torch.rand(N * N + len(ars) * len(acs) * 64, dtype=torch.float32, device="cuda")
C = torch.rand(N * N + len(crs) * len(ccs) * 64, dtype=torch.float32, device="cuda")
LA, LC = layout(ars, acs, A), layout(crs, ccs, C)
comm = costa.Comm.self(0)
steps = 5
costa.set_profiling(True)
for _ in range(steps):
    costa.transform_async(LA, LC, comm, op, al, be)
costa.synchronize(comm)
st = costa.get_stats(reset=True)
costa.set_profiling(False)
el = N * N * 4
p = costa.plan_export([LA], [LC], 0, 1)
print(json.dumps({"op": op, "edge_multiple": Q, "tiles": int(p.local_ops.size),
                  "local_launches_per_step": st["local_launches"] / steps,
                  "read_bytes": el * (2 if be != 0 else 1), "write_bytes": el,
                  "alg_bytes_per_launch": st["local_bytes"] / max(1, st["local_launches"]),
                  "kernel_ms": round(st["local_ms"] / max(1, st["local_launches"]), 4)}),
      flush=True)
