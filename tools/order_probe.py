"""Tuning probe (not product): one 'T' transform of an n x n matrix on one GPU, kernel time from
the library's own events.  Used to compare large-shape sub-tile orders (COSTA_TUNING=1 COSTA_LARGE_SORT) across
element types, block sizes and beta:
    python tools/order_probe.py DTYPE N BLOCK BETA [steps]      DTYPE in f32 f64 c64 c128
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import costa_amd as costa  # noqa: E402


OP = os.environ.get("COSTA_PROBE_OP", "T")  # op of the probe transform (tuning: N for copies)


def main():
    dt, n, b, beta = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    cd, tdt = {"f32": (costa.FLOAT, torch.float32), "f64": (costa.DOUBLE, torch.float64),
               "c64": (costa.CFLOAT, torch.complex64),
               "c128": (costa.CDOUBLE, torch.complex128)}[dt]
    costa.lib()
    comm = costa.Comm.self(0)
    es = torch.tensor([], dtype=tdt).element_size()
    pad = int(os.environ.get("COSTA_PROBE_LDPAD", "0"))  # leading-dimension padding (elements)
    ld = n + pad
    A = torch.rand(ld * n, dtype=tdt, device="cuda")
    C = torch.rand(ld * n, dtype=tdt, device="cuda")
    LA = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), ld, "C", 0,
                                   dtype=cd)
    LC = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, C.data_ptr(), ld, "C", 0,
                                   dtype=cd)
    al = 0.5 if beta != 0 else 1.0
    for _ in range(3):
        costa.transform_async(LA, LC, comm, OP, al, beta)
    costa.synchronize(comm)
    costa.set_profiling(True)
    costa.get_stats(reset=True)
    for _ in range(steps):
        costa.transform_async(LA, LC, comm, OP, al, beta)
    costa.synchronize(comm)
    st = costa.get_stats(reset=True)
    ms = st["local_ms"] / steps
    gbps = (3 if beta != 0 else 2) * n * n * es / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    extra = ""
    if st["pack_launches"]:  # COSTA_LOOPBACK=1: every tile through the exchange
        extra = "".join(f"  {k} {st[k + '_ms'] / steps:.4f} ms "
                        f"{st[k + '_bytes'] / steps / (st[k + '_ms'] / steps * 1e-3) / 1e9:7.1f} GB/s"
                        for k in ("pack", "unpack"))
    print(f"{dt} {n}^2 ld +{pad} block {b} beta {beta} sort {os.environ.get('COSTA_LARGE_SORT', '1')}: "
          f"kernel {ms:.4f} ms {gbps:8.1f} GB/s{extra}", flush=True)


if __name__ == "__main__":
    main()
