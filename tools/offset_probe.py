"""Tuning probe (not product): does the relative placement of A and C in device memory change
cfg 2's kernel time?  (Fresh processes see 0.671 or 0.698 ms for the same binary.)  A and C are
carved out of one allocation at offsets 0 and 2 GiB + delta; kernel time from the library's events.
    python tools/offset_probe.py [steps]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import costa_amd as costa  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    costa.lib()
    comm = costa.Comm.self(0)
    n, b = 16384, 256
    nbytes = n * n * 8
    pool = torch.empty(2 * nbytes + (256 << 20), dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    base_al = (base + (2 << 20) - 1) // (2 << 20) * (2 << 20)
    A = pool[base_al - base: base_al - base + nbytes].view(torch.float64)
    A.copy_(torch.rand(n * n, dtype=torch.float64, device="cuda"))
    print(f"pool base % 2MiB = {base % (2 << 20)}", flush=True)
    for delta in [0, 4096, 65536, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20, 32 << 20, 64 << 20,
                  128 << 20, 3 << 20, 6 << 20, 12 << 20, 0]:
        off = base_al - base + nbytes + delta
        C = pool[off: off + nbytes].view(torch.float64)
        LA = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), n, "C", 0)
        LC = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, C.data_ptr(), n, "C", 0)
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
        ok = torch.equal(C.view(n, n), A.view(n, n).t())
        ms = st["local_ms"] / steps
        print(f"C = A + 2 GiB + {delta >> 10:7d} KiB: kernel {ms:.4f} ms {2 * nbytes / ms / 1e6:8.1f} GB/s "
              f"{'ok' if ok else 'WRONG'}", flush=True)
        costa.release_caches()


if __name__ == "__main__":
    main()
