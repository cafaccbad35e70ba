"""Tuning probe (not product): transposing access patterns without LDS (libcosta_ceiling kinds
100 + 10 g + m: fp64 sub-tile geometry g = 64 x 128 / 32 x 256 / 16 x 512 / 128 x 64 / 256 x 32;
m 0 both sides transposed, 1 flat loads + transposed stores, 2 transposed loads + flat stores)
beside the headline transpose and the one-vector copy, per buffer pair (16384^2 fp64).
    python tools/pattern_probe.py [pairs] [pol]   (pol: kind 5 with each store cache policy,
                                                   kinds 200-205; ord: sub-tile orders, 300-305;
                                                   r6: kinds 5, 306, 400, 401)"""
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
GEO = ["64x128", "32x256", "16x512", "128x64", "256x32"]
POL = ORD = R6 = False


def main():
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    global POL
    POL = len(sys.argv) > 2 and sys.argv[2] == "pol"
    global ORD, R6
    ORD = len(sys.argv) > 2 and sys.argv[2] == "ord"
    R6 = len(sys.argv) > 2 and sys.argv[2] == "r6"
    costa.lib()
    comm = costa.Comm.self(0)
    ceil = C.CDLL(os.path.join(ROOT, "costa_amd", "lib", "libcosta_ceiling.so"))
    f = ceil.costa_ceiling_copy_ms
    f.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.POINTER(C.c_float)]

    def med(kind, a, c):
        m = (C.c_float * 10)()
        rc = f(kind, a.data_ptr(), c.data_ptr(), BYTES, N * 8, 10, m)
        return statistics.median(list(m)) if rc == 0 else float("nan")
    for k in range(pairs):
        a = torch.empty(N * N, dtype=torch.float64, device="cuda")
        c = torch.empty(N * N, dtype=torch.float64, device="cuda")
        LA = costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, a.data_ptr(), N, "C", 0)
        LC = costa.block_cyclic_layout(N, N, B, B, 1, 1, N, N, 1, 1, "R", 0, 0, c.data_ptr(), N, "C", 0)
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
        line = [f"pair {k}: transpose {ms:.4f} copy {med(4, a, c):.4f}"]
        if R6:  # the two candidates not probed before, beside kind 5
            line.append("kind 5 / XCD row-band rotation (306) / 2 KiB segments 1024 thr (400) / 512 thr (401) " +
                        " / ".join(f"{med(q, a, c):.4f}" for q in (5, 306, 400, 401)))
        elif ORD:  # kind 5's pattern with each sub-tile order
            line.append("orders band-major / band up / bands reversed / boustrophedon / band per XCD / "
                        "4 bands abreast " + " / ".join(f"{med(300 + q, a, c):.4f}" for q in range(6)))
        elif POL:  # kind 5's pattern with each store cache policy
            line.append("stores nt / default / sc1 / sc1 nt / sc0 nt / sc0 sc1 nt " +
                        " / ".join(f"{med(200 + q, a, c):.4f}" for q in range(6)))
        else:
            for g, name in enumerate(GEO):
                line.append(f"{name} " + "/".join(f"{med(100 + 10 * g + m, a, c):.4f}" for m in range(3)))
        print("  ".join(line), flush=True)
        del LA, LC, a, c
        costa.release_caches()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
