#!/usr/bin/env python3
"""What bounds the wavefront path on ragged tiles: cfg 5's geometry (fp32 16384^2 'N', A block
edges 8-96, C block edges 16-160, every block its own column-major buffer) against the same
generator with every block edge rounded to a multiple of 32 elements (128 bytes: every tile
column starts and ends on a cache line) or of 4 (16 bytes), and with edges scaled (fewer,
larger tiles), to separate the alignment of the column runs from the tile size.
    python tools/c5_align_probe.py        (GPU box)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import costa_amd as costa  # noqa: E402

N = 16384


def splits(seed, lo, hi, q, scale=1.0):
    r = np.random.default_rng(seed)
    s = [0]
    while s[-1] < N:
        e = int(round(int(r.integers(lo, hi + 1)) * scale))
        e = max(q, (e + q // 2) // q * q)
        s.append(min(N, s[-1] + e))
    return s


def layout(rs, cs, buf):
    blocks, off = [], 0
    for i in range(len(rs) - 1):
        for j in range(len(cs) - 1):
            rows, cols = rs[i + 1] - rs[i], cs[j + 1] - cs[j]
            blocks.append((buf.data_ptr() + ES * off, rows, i, j))
            off += (rows * cols + 63) // 64 * 64
    own = np.zeros((len(rs) - 1, len(cs) - 1), np.int64)
    return costa.custom_layout(len(rs) - 1, len(cs) - 1, rs, cs, own, blocks, "C", CDT), off


OP = os.environ.get("PROBE_OP", "N")  # 'T': alpha=-0.5, beta=2 (cfg 5's 'T' variant)
# PROBE_DTYPE=double: the same geometry in fp64; PROBE_FIRST=1: only the first (cfg 5) case
TDT, CDT, ES = ((torch.float64, costa.DOUBLE, 8) if os.environ.get("PROBE_DTYPE") == "double"
                else (torch.float32, costa.FLOAT, 4))
AL, BE = (1.0, 0.0) if OP == "N" else (-0.5, 2.0)


def run(q, scale=1.0, qc=None):
    qc = q if qc is None else qc  # C's edges may be rounded differently from A's
    ars, acs = splits(0xC5A1, 8, 96, q, scale), splits(0xC5A2, 8, 96, q, scale)
    crs, ccs = splits(0xC5A3, 16, 160, qc, scale), splits(0xC5A4, 16, 160, qc, scale)
    A = torch.rand(N * N + (len(ars) * len(acs)) * 64, dtype=TDT, device="cuda")
    C = torch.zeros(N * N + (len(crs) * len(ccs)) * 64, dtype=TDT, device="cuda")
    LA, _ = layout(ars, acs, A)
    LC, _ = layout(crs, ccs, C)
    comm = costa.Comm.self(0)
    for _ in range(3):
        costa.transform_async(LA, LC, comm, OP, AL, BE)
    costa.synchronize(comm)
    costa.set_profiling(True)
    costa.get_stats(reset=True)
    steps = 10
    for _ in range(steps):
        costa.transform_async(LA, LC, comm, OP, AL, BE)
    costa.synchronize(comm)
    st = costa.get_stats(reset=True)
    costa.set_profiling(False)
    p = costa.plan_export([LA], [LC], 0, 1)
    ms = st["local_ms"] / steps
    print(json.dumps({"op": OP, "edge_multiple_A": q, "edge_multiple_C": qc, "edge_scale": scale,
                      "tiles": int(p.local_ops.size),
                      "kernel_ms": round(ms, 4),
                      "GBps": round(st["local_bytes"] / steps / (ms * 1e-3) / 1e9, 1)}), flush=True)


CASES = ((1, 1.0, 1), (4, 1.0, 4), (32, 1.0, 32), (1, 1.35, 1), (1, 2.0, 1),
                     (32, 0.75, 32), (32, 1.0, 1), (1, 1.0, 32))
for q, scale, qc in CASES[:1] if os.environ.get("PROBE_FIRST") else CASES:
    run(q, scale, qc)
