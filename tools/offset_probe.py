"""Tuning probe (not product): does the headline transpose's rate depend on where A and C lie
relative to each other?  (r3-r5: one process runs cfg 2 at 0.665-0.671 ms, the next at 0.697,
while the copy of the same bytes does not move.)  One 5 GiB allocation, A at offset 0, C at
2 GiB + delta (and C first, A after it), then separate allocations as bench.py makes them; the
kernel time of 10 transforms each (library events).
    python tools/offset_probe.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import costa_amd as costa  # noqa: E402

N, B = 16384, 256
BYTES = N * N * 8


def kernel_ms(pa, pc, comm, steps=10):
    LA = costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, pa, N, "C", 0)
    LC = costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, pc, N, "C", 0)
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
    costa.release_caches()
    return st["local_ms"] / steps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    costa.lib()
    comm = costa.Comm.self(0)
    deltas = [0, 4096, 65536, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20, 64 << 20, 256 << 20, 1 << 30]
    pool = torch.empty(2 * BYTES + (1 << 30), dtype=torch.uint8, device="cuda")
    base = pool.data_ptr()
    for r in range(reps):
        for d in deltas:
            ms = kernel_ms(base, base + BYTES + d, comm)
            ms2 = kernel_ms(base + BYTES + d, base, comm)  # roles swapped
            print(f"rep {r} delta {d >> 10:8d} KiB: A then C {ms:.4f} ms   C then A {ms2:.4f} ms", flush=True)
    del pool
    torch.cuda.empty_cache()
    for r in range(4):  # separate allocations, as bench.py
        A = torch.empty(N * N, dtype=torch.float64, device="cuda")
        C = torch.empty(N * N, dtype=torch.float64, device="cuda")
        ms = kernel_ms(A.data_ptr(), C.data_ptr(), comm)
        print(f"separate allocations {r}: A {A.data_ptr():#x} C {C.data_ptr():#x}: {ms:.4f} ms", flush=True)
        del A, C
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
