"""Tuning probe (not product): p?gemr2d-style copies ('N') into destination columns off the
64-byte grid (ldc = n + pad), 16384^2, 256^2 blocks, one rank; kernel time from the library's own
events, result checked (C == A, padding untouched).  Run once per library setting, e.g. with
COSTA_TUNING=1 COSTA_COPY_GRANULE=1 (engine.cpp granule_split) against the default.
    python tools/copy_pad_probe.py [steps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import costa_amd as costa  # noqa: E402

CASES = [  # (dtype, lda pad, ldc pad, beta)
    (costa.DOUBLE, 0, 0, 0.0), (costa.DOUBLE, 0, 1, 0.0), (costa.DOUBLE, 0, 2, 0.0),
    (costa.DOUBLE, 0, 3, 0.0), (costa.DOUBLE, 0, 8, 0.0), (costa.DOUBLE, 1, 1, 0.0),
    (costa.DOUBLE, 0, 2, 0.5), (costa.FLOAT, 0, 0, 0.0), (costa.FLOAT, 0, 1, 0.0),
    (costa.FLOAT, 0, 4, 0.0), (costa.FLOAT, 0, 8, 0.0), (costa.FLOAT, 0, 4, 0.5),
    (costa.INT32, 0, 3, 0.0),
]


def run(dtype, pa, pc, beta, steps, comm, n=16384, b=256):
    tdt = {costa.DOUBLE: torch.float64, costa.FLOAT: torch.float32, costa.INT32: torch.int32}[dtype]
    lda, ldc = n + pa, n + pc
    if tdt == torch.int32:
        A = torch.randint(-1000, 1000, (n, lda), dtype=tdt, device="cuda")
    else:
        A = torch.rand(n, lda, dtype=tdt, device="cuda")
    C = torch.full((n, ldc), 7, dtype=tdt, device="cuda")
    es = A.element_size()
    LA = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), lda, "C", 0,
                                   dtype=dtype)
    LC = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, C.data_ptr(), ldc, "C", 0,
                                   dtype=dtype)
    al = 1 if tdt == torch.int32 else 1.0
    costa.transform(LA, LC, comm, "N", al, 0 * beta)
    ok = torch.equal(C[:, :n], A[:, :n]) and bool((C[:, n:] == 7).all())
    for _ in range(3):
        costa.transform_async(LA, LC, comm, "N", al, beta)
    costa.synchronize(comm)
    costa.set_profiling(True)
    costa.get_stats(reset=True)
    for _ in range(steps):
        costa.transform_async(LA, LC, comm, "N", al, beta)
    costa.synchronize(comm)
    st = costa.get_stats(reset=True)
    costa.set_profiling(False)
    ms = st["local_ms"] / steps
    gbps = (2 + (beta != 0)) * n * n * es / (ms * 1e-3) / 1e9
    name = {costa.DOUBLE: "fp64", costa.FLOAT: "fp32", costa.INT32: "i32"}[dtype]
    print(f"{name} 'N' lda +{pa} ldc +{pc} beta {beta}: kernel {ms:.4f} ms  {gbps:8.1f} GB/s  "
          f"launches/step {st['local_launches'] / steps:.0f}  {'ok' if ok else 'WRONG'}", flush=True)
    del A, C, LA, LC
    costa.release_caches()
    torch.cuda.empty_cache()
    return ok


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    costa.lib()
    comm = costa.Comm.self(0)
    bad = 0
    for c in CASES:
        bad += not run(*c, steps, comm)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
