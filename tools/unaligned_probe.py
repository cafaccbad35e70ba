"""Tuning probe (not product): large tiles whose columns are not 16-byte aligned.

A ScaLAPACK matrix with an odd lld (fp64) or lld % 4 != 0 (fp32) has tiles the large shape
cannot load with 16-byte vectors; the engine sends those ops either through the large shape's
guarded path (above kUnalignedWaveCap sub-tiles) or cuts them into wavefront pieces. This times
the 16384^2 'T' transpose (alpha=1, beta=0) at aligned and unaligned lld, 256^2 and 128^2 blocks,
fp64 and fp32, kernel time from the library's own events.
    python tools/unaligned_probe.py [steps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import costa_amd as costa  # noqa: E402


def run(dtype, n, b, lld, steps, comm, lldc=None):
    lldc = lldc or lld
    tdt = {costa.DOUBLE: torch.float64, costa.FLOAT: torch.float32}[dtype]
    es = torch.tensor([], dtype=tdt).element_size()
    A = torch.rand(lld * n, dtype=tdt, device="cuda")
    C = torch.zeros(lldc * n, dtype=tdt, device="cuda")
    LA = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), lld, "C", 0,
                                   dtype=dtype)
    LC = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, C.data_ptr(), lldc, "C", 0,
                                   dtype=dtype)
    costa.transform(LA, LC, comm, "T", 1.0, 0.0)
    ok = torch.equal(C.view(n, lldc)[:, :n], A.view(n, lld)[:, :n].t())
    for _ in range(3):
        costa.transform_async(LA, LC, comm, "T", 1.0, 0.0)
    costa.synchronize(comm)
    costa.set_profiling(True)
    costa.get_stats(reset=True)
    for _ in range(steps):
        costa.transform_async(LA, LC, comm, "T", 1.0, 0.0)
    costa.synchronize(comm)
    st = costa.get_stats(reset=True)
    costa.set_profiling(False)
    ms = st["local_ms"] / steps
    gbps = 2 * n * n * es / (ms * 1e-3) / 1e9
    name = "fp64" if dtype == costa.DOUBLE else "fp32"
    print(f"{name} {n}^2 blocks {b}^2 lld {lld}/{lldc}: kernel {ms:.4f} ms  {gbps:8.1f} GB/s  "
          f"launches/step {st['local_launches'] / steps:.0f}  {'ok' if ok else 'WRONG'}", flush=True)
    del A, C, LA, LC
    costa.release_caches()
    torch.cuda.empty_cache()


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    costa.lib()
    comm = costa.Comm.self(0)
    n = 16384
    if len(sys.argv) > 2 and sys.argv[2] == "sides":  # one side misaligned at a time
        for dtype, odd in ((costa.DOUBLE, 16385), (costa.FLOAT, 16386)):
            for la, lc in ((16384, 16384), (odd, 16384), (16384, odd), (odd, odd)):
                run(dtype, n, 256, la, steps, comm, lc)
        run(costa.FLOAT, n, 256, 16385, steps, comm, 16385)
        return
    for dtype, llds in ((costa.DOUBLE, (16384, 16385)), (costa.FLOAT, (16384, 16385, 16386))):
        for b in (512, 256, 128):
            for lld in llds:
                run(dtype, n, b, lld, steps, comm)


if __name__ == "__main__":
    main()
