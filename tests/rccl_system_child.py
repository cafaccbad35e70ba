"""Child process of test_gpu_rccl_system.py: the exchange on the RCCL that C, C++ and ScaLAPACK
callers get (/opt/rocm/lib/librccl.so.1, which libcosta_amd.so links), not torch's bundled copy.

torch is never imported here (COSTA_NO_TORCH=1), so the loader binds the system HIP runtime and
RCCL; device memory comes from hipMalloc through ctypes.  With COSTA_LOOPBACK=1 every tile of a
one-rank transform goes PACK -> ncclSend/ncclRecv to self -> UNPACK (engine.hpp
loopback_exchange), so the RCCL group of the reference's exchange_async (transform.cpp:46-128)
runs on this library:
  * every single-rank golden case, against the reference's outputs bit for bit;
  * 12288^2 fp64 'T' (a 1.2 GB package: an unchunked self send/recv of it lost its second half
    on torch's RCCL), moved in the default 256 MiB pieces, or in pieces of the
    largest size the library allows when COSTA_MAX_MSG_BYTES asks for more;
  * 23168^2 fp64 'N' with 128^2 blocks: a 4.29 GB package, BASELINE cfg 3's per-peer size, in
    17 pieces over 4 exchange rounds.
Prints 'COSTA_RCCL <version> <library path>' and a final 'OK <cases>' or 'FAIL ...' lines."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402

import costa_amd as costa  # noqa: E402
import oracle  # noqa: E402
from cases import all_cases  # noqa: E402
from golden_io import load, matches  # noqa: E402

H2D, D2H = 1, 2


class Hip:
    def __init__(self):
        costa.lib()  # binds libamdhip64.so.7 (the system runtime) first
        self.L = C.CDLL("libamdhip64.so.7")
        self.L.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        self.L.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self.L.hipFree.argtypes = [C.c_void_p]
        self.L.hipDeviceSynchronize.argtypes = []

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        p = C.c_void_p()
        assert self.L.hipMalloc(C.byref(p), max(arr.nbytes, 16)) == 0
        assert self.L.hipMemcpy(p, arr.ctypes.data, arr.nbytes, H2D) == 0
        return p.value

    def download(self, p, like):
        out = np.empty_like(like)
        assert self.L.hipDeviceSynchronize() == 0
        assert self.L.hipMemcpy(out.ctypes.data, p, out.nbytes, D2H) == 0
        return out

    def free(self, p):
        self.L.hipFree(p)


def rccl_path():
    for line in open("/proc/self/maps"):
        if "librccl" in line:
            return line.split()[-1]
    return "?"


def main():
    assert os.environ.get("COSTA_LOOPBACK") == "1"
    hip = Hip()
    comm = costa.Comm.self(0)  # the one-rank RCCL communicator is created here
    assert "torch" not in sys.modules, "torch was imported: its RCCL would be the one bound"
    v = costa.rccl_version()
    print("COSTA_RCCL", f"{v // 10000}.{v // 100 % 100}.{v % 100}", rccl_path(), flush=True)
    costa.set_profiling(True)
    costa.get_stats(reset=True)
    bad, n = [], 0
    for case in all_cases():
        if case.P != 1:
            continue
        n += 1
        host = [case.inputs(k, 0) for k in range(len(case.pairs))]
        dev = [(hip.upload(a), hip.upload(c)) for a, c in host]
        As = [case.layout_A(k, 0, dev[k][0]) for k in range(len(case.pairs))]
        Cs = [case.layout_C(k, 0, dev[k][1]) for k in range(len(case.pairs))]
        eff = [case.effective(k) for k in range(len(case.pairs))]
        costa.transform_batch(As, Cs, comm, [e[0] for e in eff], [e[1] for e in eff],
                              [e[2] for e in eff])
        fx = load(case.name)
        for k in range(len(case.pairs)):
            if not matches(fx, f"C{k}_r0", hip.download(dev[k][1], host[k][1])):
                bad.append(f"{case.name} C{k}")
        for a, c in dev:
            hip.free(a)
            hip.free(c)
    m = 12288
    a = np.random.default_rng(12288).standard_normal(m * m)
    pa, pc = hip.upload(a), hip.upload(np.zeros(m * m))
    LA = costa.block_cyclic_layout(m, m, 256, 256, 1, 1, m, m, 1, 1, "R", 0, 0, pa, m, "C", 0)
    LC = costa.block_cyclic_layout(m, m, 256, 256, 1, 1, m, m, 1, 1, "R", 0, 0, pc, m, "C", 0)
    costa.transform(LA, LC, comm, "T", 1.0, 0.0)
    got = hip.download(pc, a)
    if not np.array_equal(got.reshape(m, m), a.reshape(m, m).T):
        half = got.reshape(m, m)[m // 2:]
        bad.append(f"{m}^2 fp64 T (second half zero: {bool((half == 0).all())})")
    hip.free(pa)
    hip.free(pc)
    # a BASELINE cfg 3-sized package: 23168^2 fp64 'N' (128^2 blocks), 4.29 GB to "the peer" =
    # 17 pieces of <= 256 MiB in 4 exchange rounds (engine.cpp round_range / max_message_bytes)
    m = 23168
    a = np.arange(m * m, dtype=np.float64)
    pa, pc = hip.upload(a), hip.upload(np.zeros(m * m))
    LA = costa.block_cyclic_layout(m, m, 128, 128, 1, 1, m, m, 1, 1, "R", 0, 0, pa, m, "C", 0)
    LC = costa.block_cyclic_layout(m, m, 128, 128, 1, 1, m, m, 1, 1, "R", 0, 0, pc, m, "C", 0)
    costa.transform(LA, LC, comm, "N", 1.0, 0.0)
    got = hip.download(pc, a)
    if not np.array_equal(got, a):
        bad.append(f"{m}^2 fp64 N: {int((got != a).sum())} elements differ")
    hip.free(pa)
    hip.free(pc)
    st = costa.get_stats()
    if st["pack_launches"] < n + 1 or st["unpack_launches"] < n + 1 or st["local_launches"]:
        bad.append(f"not every case went through the exchange: {st}")
    for b in bad:
        print("FAIL", b)
    print("OK" if not bad else "BAD", n + 2)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
