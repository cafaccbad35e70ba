"""Probe (not a test): COSTA_LOOPBACK=1 transforms of m x m fp64 'T' at several sizes and call
counts; prints which combinations produce C == A^T and, for failures, where C differs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import costa_amd as costa  # noqa: E402

comm = costa.Comm.self(0)
for m, calls in [(8192, 1), (11584, 1), (12288, 1), (16384, 2)]:
    A = torch.rand(m * m, dtype=torch.float64, device="cuda")
    Cm = torch.zeros(m * m, dtype=torch.float64, device="cuda")
    LA = costa.block_cyclic_layout(m, m, 256, 256, 1, 1, m, m, 1, 1, "R", 0, 0, A.data_ptr(), m, "C", 0)
    LC = costa.block_cyclic_layout(m, m, 256, 256, 1, 1, m, m, 1, 1, "R", 0, 0, Cm.data_ptr(), m, "C", 0)
    for _ in range(calls):
        costa.transform(LA, LC, comm, "T", 1.0, 0.0)
    torch.cuda.synchronize()
    ok = torch.equal(Cm.view(m, m), A.view(m, m).t())
    msg = ""
    if not ok:
        d = (Cm.view(m, m) != A.view(m, m).t())
        rows = d.any(1).nonzero().flatten()
        cols = d.any(0).nonzero().flatten()
        zero = (Cm == 0).sum().item()
        msg = (f" bad={d.sum().item()} rows {rows.min().item()}..{rows.max().item()} "
               f"cols {cols.min().item()}..{cols.max().item()} zeros={zero}")
    print(f"m={m} calls={calls} ok={ok}{msg}", flush=True)
    del A, Cm, LA, LC
    costa.release_caches()
