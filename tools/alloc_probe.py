"""Tuning probe (not product): does the headline transpose's placement mode (r5, DESIGN.md §3c: the
destination buffer's physical pages decide between ~0.66 and ~0.70 ms) follow how the destination
was allocated?  One source A (torch), K destinations per allocation kind:
    torch       torch's caching allocator (what bench.py and most callers use)
    malloc      hipMalloc
    contig      hipExtMallocWithFlags(hipDeviceMallocContiguous): physically contiguous
Per destination: the transpose's kernel time (library events, 10 calls, 2 rounds).
    python tools/alloc_probe.py [K] [kinds]
    python tools/alloc_probe.py pairs [K]   K (A, C) pairs from torch's allocator, then K
                                            physically contiguous ones, alternating rounds"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import costa_amd as costa  # noqa: E402

N, B = 16384, 256
BYTES = N * N * 8


class Contig:
    """a physically contiguous fp64 device buffer (hipExtMallocWithFlags) viewed as a tensor"""
    def __init__(self, nbytes):
        hip = C.CDLL("libamdhip64.so")
        hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
        p = C.c_void_p()
        assert hip.hipExtMallocWithFlags(C.byref(p), nbytes, 0x4) == 0
        self.__cuda_array_interface__ = {"shape": (nbytes // 8,), "typestr": "<f8", "data": (p.value, False),
                                         "strides": None, "version": 2}
        self.t = torch.as_tensor(self, device="cuda")


def timed(LA, LC, comm):
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
    return ms


def pairs(k):
    comm = costa.Comm.self(0)
    sets, keep = {}, []
    for kind in ("torch", "pool"):
        bufs = []
        for i in range(k):
            if kind == "pool":
                keep.append((Contig(BYTES), Contig(BYTES)))
                a, c = keep[-1][0].t, keep[-1][1].t
            else:
                a = torch.empty(N * N, dtype=torch.float64, device="cuda")
                c = torch.empty(N * N, dtype=torch.float64, device="cuda")
            a.copy_(torch.arange(N * N, dtype=torch.float64, device="cuda"))
            bufs.append((a, c))
        sets[kind] = bufs
    for r in range(2):
        for kind, bufs in sets.items():
            for i, (a, c) in enumerate(bufs):
                LA = costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, a.data_ptr(), N, "C", 0)
                LC = costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, c.data_ptr(), N, "C", 0)
                ms = timed(LA, LC, comm)
                ok = torch.equal(c.view(N, N), a.view(N, N).T)
                print(f"round {r} {kind} pair {i}: transpose {ms:.4f} ms  {'ok' if ok else 'MISMATCH'}  "
                      f"(A 0x{a.data_ptr():x} C 0x{c.data_ptr():x})", flush=True)
                del LA, LC
                costa.release_caches()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "pairs":
        costa.lib()
        return pairs(int(sys.argv[2]) if len(sys.argv) > 2 else 4)
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    kinds = sys.argv[2].split(",") if len(sys.argv) > 2 else ["torch", "malloc", "contig"]
    costa.lib()
    hip = C.CDLL("libamdhip64.so")
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    hip.hipFree.argtypes = [C.c_void_p]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    comm = costa.Comm.self(0)
    A = torch.empty(N * N, dtype=torch.float64, device="cuda")
    A.copy_(torch.arange(N * N, dtype=torch.float64, device="cuda"))
    LA = costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, A.data_ptr(), N, "C", 0)
    dsts = []
    for kind in kinds:
        for i in range(k):
            if kind == "torch":
                t = torch.empty(N * N, dtype=torch.float64, device="cuda")
                dsts.append((kind, i, t.data_ptr(), t))
                continue
            p = C.c_void_p()
            rc = (hip.hipMalloc(C.byref(p), BYTES) if kind == "malloc"
                  else hip.hipExtMallocWithFlags(C.byref(p), BYTES, 0x4))
            if rc != 0:
                print(f"{kind} {i}: allocation failed ({rc})", flush=True)
                continue
            dsts.append((kind, i, p.value, None))
    Aref = A.view(N, N)
    for r in range(2):
        for kind, i, ptr, _ in dsts:
            LC = costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, ptr, N, "C", 0)
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
            # check a row of the result: C(j, i) = A(i, j), C column-major with ld N
            Ct = torch.empty(N, dtype=torch.float64, device="cuda")
            hip.hipMemcpy(C.c_void_p(Ct.data_ptr()), C.c_void_p(ptr + 8 * N * 77), 8 * N, 3)
            ok = torch.equal(Ct, Aref[:, 77].contiguous())
            print(f"round {r} {kind} {i}: transpose {ms:.4f} ms  {'ok' if ok else 'MISMATCH'}  "
                  f"(dst 0x{ptr:x})", flush=True)
            costa.release_caches()
    for kind, i, ptr, _ in dsts:
        if kind != "torch":
            hip.hipFree(C.c_void_p(ptr))


if __name__ == "__main__":
    main()
