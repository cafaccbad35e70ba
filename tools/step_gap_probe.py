#!/usr/bin/env python3
"""Probe (not product): where does the per-step time above the kernel go on cfg 2?

Times K async steps of the bench's cfg 2 transform with the phase-timing events on and off,
interleaved, and reports ms/step against the tile kernel's own event time.
    python tools/step_gap_probe.py [K] [reps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import costa_amd as costa  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 50
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
costa.lib()
torch.cuda.set_device(0)
comm = costa.Comm.self(0)
n, b = 16384, 256
A = torch.rand(n * n, dtype=torch.float64, device="cuda")
C = torch.zeros(n * n, dtype=torch.float64, device="cuda")
LA = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), n, "C", 0)
LC = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, C.data_ptr(), n, "C", 0)
for _ in range(5):
    costa.transform(LA, LC, comm, "T", 1.0, 0.0)
torch.cuda.synchronize()
assert torch.equal(C.view(n, n), A.view(n, n).t())


def run(profile: bool):
    costa.set_profiling(profile)
    costa.get_stats(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        costa.transform_async(LA, LC, comm, "T", 1.0, 0.0)
    costa.synchronize(comm)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = costa.get_stats(reset=True)
    costa.set_profiling(False)
    return el / K * 1e3, st["local_ms"] / K if profile else None


for r in range(reps):
    for prof in (True, False):
        ms, kms = run(prof)
        print(f"rep{r} K={K} events={'on ' if prof else 'off'} ms/step {ms:.4f}"
              + (f" kernel {kms:.4f} gap {ms - kms:.4f}" if kms else ""), flush=True)
