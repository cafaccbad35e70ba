"""Tuning probe (not product): copy lists on the large shape. 16384^2 'N' (layouts with the same
blocks, every tile a local copy), 256^2 blocks, per element type, alpha=1 beta=0 (bit copy) and
alpha=0.5 beta=1.5 (C read); kernel time from the library's own events.
    python tools/copy_probe.py [steps] [block edges, comma-separated] [types, comma-separated]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import costa_amd as costa  # noqa: E402

TYPES = [("f32", costa.FLOAT, torch.float32), ("f64", costa.DOUBLE, torch.float64),
         ("c64", costa.CFLOAT, torch.complex64), ("c128", costa.CDOUBLE, torch.complex128)]


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    blocks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [256]
    types = sys.argv[3].split(",") if len(sys.argv) > 3 else [t[0] for t in TYPES]
    costa.lib()
    comm = costa.Comm.self(0)
    n = 16384
    for (name, code, tdt), b in [(t, b) for t in TYPES if t[0] in types for b in blocks]:
        for al, be in ((1.0, 0.0), (0.5, 1.5)):
            A = torch.rand(n * n, dtype=tdt, device="cuda")
            C = torch.rand(n * n, dtype=tdt, device="cuda")
            LA = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), n, "C", 0,
                                           dtype=code)
            LC = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, C.data_ptr(), n, "C", 0,
                                           dtype=code)
            C0 = C.clone() if be != 0 else None
            costa.transform(LA, LC, comm, "N", al, be)
            ok = torch.equal(C, A) if be == 0 else torch.allclose(C, be * C0 + al * A, rtol=1e-5, atol=1e-5)
            del C0
            for _ in range(2):
                costa.transform_async(LA, LC, comm, "N", al, be)
            costa.synchronize(comm)
            costa.set_profiling(True)
            costa.get_stats(reset=True)
            for _ in range(steps):
                costa.transform_async(LA, LC, comm, "N", al, be)
            costa.synchronize(comm)
            st = costa.get_stats(reset=True)
            costa.set_profiling(False)
            ms = st["local_ms"] / steps
            gbps = st["local_bytes"] / steps / (ms * 1e-3) / 1e9
            print(f"{name} copy 16384^2 {b}^2 blocks alpha={al} beta={be}: kernel {ms:.4f} ms {gbps:8.1f} GB/s "
                  f"{'ok' if ok else 'WRONG'}", flush=True)
            del A, C, LA, LC
            costa.release_caches()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
