"""Tuning probe (not product): several builds of libcosta_amd.so loaded side by side in ONE
process (RTLD_LOCAL, raw C ABI), timed on the SAME buffers -- the headline's rate depends on where
the destination buffer lies physically (r5, tools/pairs_probe.py), so builds compared in separate
processes see different placements.  K pairs of 2 GiB buffers; per pair and build the kernel time
of 10 stream-ordered transforms (the library's own events), C checked against A^T once.
    python tools/libs_probe.py <pairs> <label=path.so> [<label=path.so> ...]
(beta != 0 runs are timed only: C changes every call)"""
import ctypes as C
import os
import sys

import torch

# PROBE_DT (f64 | f32 | c64 | c128), PROBE_N, PROBE_B, PROBE_BETA: other headline-like geometries
DT = os.environ.get("PROBE_DT", "f64")
N, B = int(os.environ.get("PROBE_N", "16384")), int(os.environ.get("PROBE_B", "256"))
BETA = float(os.environ.get("PROBE_BETA", "0"))
OP = os.environ.get("PROBE_OP", "T")  # N: the copy
CODE, TDT = {"f32": (0, torch.float32), "f64": (1, torch.float64), "c64": (2, torch.complex64),
             "c128": (3, torch.complex128)}[DT]


class Stats(C.Structure):  # costa_stats_t (include/costa_hip.h)
    _fields_ = [(k, C.c_double) for k in ("pack_ms", "local_ms", "unpack_ms", "exchange_ms", "h2d_ms", "d2h_ms")] + \
               [(k, C.c_int64) for k in ("pack_launches", "local_launches", "unpack_launches", "pack_bytes",
                                         "local_bytes", "unpack_bytes", "transforms", "plan_hits", "plan_misses",
                                         "host_groups", "device_plans")] + \
               [("plan_ms", C.c_double), ("host_direct", C.c_int64), ("host_direct_groups", C.c_int64)]


class Lib:
    def __init__(self, path):
        self.L = C.CDLL(path, mode=C.RTLD_LOCAL)
        vp, i, c = C.c_void_p, C.c_int, C.c_char
        self.L.costa_hip_block_cyclic_layout.argtypes = [i, i, i, i, i, i, i, i, i, i, i, c, i, i, vp, i, c, i,
                                                         C.POINTER(vp)]
        self.L.costa_hip_comm_self.argtypes = [i, C.POINTER(vp)]
        self.L.costa_hip_transform_async.argtypes = [vp, vp, c, vp, vp, vp, vp]
        self.L.costa_hip_synchronize.argtypes = [vp]
        self.L.costa_hip_get_stats.argtypes = [C.POINTER(Stats), i]
        self.comm = vp()
        assert self.L.costa_hip_comm_self(0, C.byref(self.comm)) == 0
        E = {0: 4, 1: 8, 2: 8, 3: 16}[CODE]
        self.alpha = (C.c_char * E)()
        self.beta = (C.c_char * E)()
        import struct
        fmt = {0: "f", 1: "d", 2: "ff", 3: "dd"}[CODE]
        av = (1.0 if BETA == 0 else 0.5,) + ((0.0,) if CODE >= 2 else ())
        bv = (BETA,) + ((0.0,) if CODE >= 2 else ())
        C.memmove(self.alpha, struct.pack(fmt, *av), E)
        C.memmove(self.beta, struct.pack(fmt, *bv), E)

    def layout(self, ptr):
        h = C.c_void_p()
        rc = self.L.costa_hip_block_cyclic_layout(CODE, N, N, B, B, 1, 1, N, N, 1, 1, b"R", 0, 0, C.c_void_p(ptr), N,
                                                  b"C", 0, C.byref(h))
        assert rc == 0
        return h

    def ms(self, LA, LC, steps=10):
        def run(k):
            for _ in range(k):
                assert self.L.costa_hip_transform_async(LA, LC, OP.encode(), self.alpha, self.beta,
                                                        self.comm, None) == 0
            assert self.L.costa_hip_synchronize(self.comm) == 0
        run(2)
        st = Stats()
        self.L.costa_hip_set_profiling(1)
        self.L.costa_hip_get_stats(C.byref(st), 1)
        run(steps)
        self.L.costa_hip_get_stats(C.byref(st), 1)
        self.L.costa_hip_set_profiling(0)
        return st.local_ms / steps


class Contig:
    """a physically contiguous device buffer (hipExtMallocWithFlags) viewed as a torch tensor"""
    hip = None

    def __init__(self, nbytes, dt):
        if Contig.hip is None:
            Contig.hip = C.CDLL("libamdhip64.so")
            Contig.hip.hipExtMallocWithFlags.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
        p = C.c_void_p()
        assert Contig.hip.hipExtMallocWithFlags(C.byref(p), nbytes, 4) == 0
        self.ptr = p.value
        ts = {torch.float32: "<f4", torch.float64: "<f8", torch.complex64: "<c8", torch.complex128: "<c16"}[dt]
        self.__cuda_array_interface__ = {"shape": (nbytes // torch.empty(0, dtype=dt).element_size(),),
                                         "typestr": ts, "data": (self.ptr, False), "strides": None, "version": 2}
        self.t = torch.as_tensor(self, device="cuda")


def main():
    pairs = int(sys.argv[1])
    libs = []
    for a in sys.argv[2:]:
        lab, _, path = a.partition("=")
        libs.append((lab, Lib(path)))
    # PROBE_ALLOC=mix: odd pairs in physically contiguous memory (hipDeviceMallocContiguous), so
    # that both placement modes show up among the pairs (r5, tools/alloc_probe.py)
    bufs, keep = [], []
    for k in range(pairs):
        if os.environ.get("PROBE_ALLOC") == "mix" and k % 2:
            a, c = Contig(N * N * torch.empty(0, dtype=TDT).element_size(), TDT), \
                Contig(N * N * torch.empty(0, dtype=TDT).element_size(), TDT)
            keep += [a, c]
            a, c = a.t, c.t
            a.copy_(torch.rand(N * N, dtype=TDT, device="cuda"))
            c.zero_()
        else:
            a, c = torch.rand(N * N, dtype=TDT, device="cuda"), torch.zeros(N * N, dtype=TDT, device="cuda")
        bufs.append((a, c))
    print("pair  " + "  ".join(f"{lab:>10s}" for lab, _ in libs), flush=True)
    for k, (a, c) in enumerate(bufs):
        row = []
        for lab, lib in libs:
            LA, LC = lib.layout(a.data_ptr()), lib.layout(c.data_ptr())
            row.append(lib.ms(LA, LC))
            torch.cuda.synchronize()
            if BETA == 0:
                want = a.view(N, N) if OP == "N" else a.view(N, N).t()
                assert torch.equal(c.view(N, N), want), f"{lab}: wrong result"
            c.zero_()
        print(f"{k:4d}  " + "  ".join(f"{x:10.4f}" for x in row), flush=True)


if __name__ == "__main__":
    main()
