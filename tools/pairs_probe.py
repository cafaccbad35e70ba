"""Tuning probe (not product): the headline transpose on K pairs of separately allocated 2 GiB
buffers in one process (r5: its rate depends on where the driver places the buffers physically --
the same virtual addresses ran 0.665 or 0.70 ms after a reallocation -- while the copy of the same
bytes does not move).  Per pair: the transpose's kernel time (library events, 10 calls) and the
one-vector strided copy (libcosta_ceiling kind 4) and the transpose's access pattern without LDS
(kind 5).  Under rocprofv3 --pmc the dispatches can be
split by duration into the two modes.
    python tools/pairs_probe.py [pairs] [rounds]
    python tools/pairs_probe.py cross [n]      n A x n C buffers, every combination"""
import ctypes as C
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import costa_amd as costa  # noqa: E402

N, B = 16384, 256
BYTES = N * N * 8


def cross(n):
    """n A buffers x n C buffers: every combination's transpose time (which side's placement
    decides the mode)"""
    comm = costa.Comm.self(0)
    As = [torch.empty(N * N, dtype=torch.float64, device="cuda") for _ in range(n)]
    Cs = [torch.empty(N * N, dtype=torch.float64, device="cuda") for _ in range(n)]
    LAs = [costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, a.data_ptr(), N, "C", 0) for a in As]
    LCs = [costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, c.data_ptr(), N, "C", 0) for c in Cs]
    print("rows: A buffer, columns: C buffer (kernel ms)")
    for i, LA in enumerate(LAs):
        line = []
        for LC in LCs:
            for _ in range(2):
                costa.transform_async(LA, LC, comm, "T", 1.0, 0.0)
            costa.synchronize(comm)
            costa.set_profiling(True)
            costa.get_stats(reset=True)
            for _ in range(10):
                costa.transform_async(LA, LC, comm, "T", 1.0, 0.0)
            costa.synchronize(comm)
            line.append(costa.get_stats(reset=True)["local_ms"] / 10)
            costa.set_profiling(False)
            costa.release_caches()
        print(f"A{i}: " + " ".join(f"{x:.4f}" for x in line), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "cross":
        costa.lib()
        return cross(int(sys.argv[2]) if len(sys.argv) > 2 else 4)
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    costa.lib()
    comm = costa.Comm.self(0)
    ceil = C.CDLL(os.path.join(ROOT, "costa_amd", "lib", "libcosta_ceiling.so"))
    f = ceil.costa_ceiling_copy_ms
    f.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_float)]
    bufs = [(torch.empty(N * N, dtype=torch.float64, device="cuda"),
             torch.empty(N * N, dtype=torch.float64, device="cuda")) for _ in range(pairs)]
    lay = [(costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, a.data_ptr(), N, "C", 0),
            costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, c.data_ptr(), N, "C", 0))
           for a, c in bufs]
    for r in range(rounds):
        for k, ((a, c), (LA, LC)) in enumerate(zip(bufs, lay)):
            for _ in range(2):
                costa.transform_async(LA, LC, comm, "T", 1.0, 0.0)
            costa.synchronize(comm)
            costa.set_profiling(True)
            costa.get_stats(reset=True)
            for _ in range(10):
                costa.transform_async(LA, LC, comm, "T", 1.0, 0.0)
            costa.synchronize(comm)
            ms = costa.get_stats(reset=True)["local_ms"] / 10
            costa.set_profiling(False)
            cm = (C.c_float * 10)()
            f(4, a.data_ptr(), c.data_ptr(), BYTES, N * 8, 10, cm)
            pm = (C.c_float * 10)()  # the transpose's access pattern without LDS (ceiling.hip kind 5)
            rc = f(5, a.data_ptr(), c.data_ptr(), BYTES, N * 8, 10, pm)
            pat = f"{statistics.median(list(pm)):.4f}" if rc == 0 else f"rc {rc}"
            qm = (C.c_float * 10)()  # the same for 128 x 128 sub-tiles (kind 6)
            rc = f(6, a.data_ptr(), c.data_ptr(), BYTES, N * 8, 10, qm)
            pat += f"  pattern128(kind 6) {statistics.median(list(qm)):.4f}" if rc == 0 else f"  rc6 {rc}"
            for kd, lab in ((7, "tr-loads"), (8, "tr-stores")):
                hm = (C.c_float * 10)()
                rc = f(kd, a.data_ptr(), c.data_ptr(), BYTES, N * 8, 10, hm)
                pat += f"  {lab}(kind {kd}) {statistics.median(list(hm)):.4f}" if rc == 0 else f"  rc{kd} {rc}"
            print(f"round {r} pair {k}: transpose {ms:.4f} ms  copy(kind 4) {statistics.median(list(cm)):.4f} ms"
                  f"  pattern(kind 5) {pat} ms", flush=True)


if __name__ == "__main__":
    main()
