"""Child process of test_gpu_loopback.py (run with COSTA_LOOPBACK=1 or 2): every single-rank
golden case, a 12288^2 fp64 'T' case and a 6144^2 alpha, beta one with 80^2 blocks (several
exchange rounds, merged tiles) go through PACK -> ncclSend/ncclRecv to self -> UNPACK
(mode 2: half of the tiles, the rest through the concurrent LOCAL launch), then a loop of
stream-ordered async transforms with A updated on torch's stream between them, then the golden
cases and a 3000 x 2500 'T' alpha/beta case from host memory through both host staging schemes
(pipelined: pack groups gathered into the send buffer, unpack groups scattered back), and again
from page-locked memory (direct groups: source rectangles DMA'd up and packed on the GPU, unpack
kernels writing target rectangles that are DMA'd back).  Prints 'DIRECT <groups>'.
Prints one line per failure and a final 'OK <cases> <pack> <unpack> <local launches>'."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import costa_amd as costa  # noqa: E402
import oracle  # noqa: E402
from cases import all_cases  # noqa: E402
from golden_io import load, matches  # noqa: E402


def dev(arr):
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy()).cuda()


def pinned(x, keep):
    """a page-locked copy of numpy array x (torch's pinned allocator = hipHostMalloc); the
    owning tensor is kept in `keep`"""
    t = torch.empty(max(1, x.nbytes), dtype=torch.uint8, pin_memory=True)
    a = t.numpy()[:x.nbytes].view(x.dtype)
    a[:] = x
    keep.append(t)
    return a


def main():
    assert os.environ.get("COSTA_LOOPBACK") in ("1", "2")
    comm = costa.Comm.self(0)
    costa.set_profiling(True)
    costa.get_stats(reset=True)
    bad, n = [], 0
    for case in all_cases():
        if case.P != 1:
            continue
        n += 1
        bufs = [tuple(dev(x) for x in case.inputs(k, 0)) for k in range(len(case.pairs))]
        As = [case.layout_A(k, 0, bufs[k][0].data_ptr()) for k in range(len(case.pairs))]
        Cs = [case.layout_C(k, 0, bufs[k][1].data_ptr()) for k in range(len(case.pairs))]
        eff = [case.effective(k) for k in range(len(case.pairs))]
        costa.transform_batch(As, Cs, comm, [e[0] for e in eff], [e[1] for e in eff],
                              [e[2] for e in eff])
        fx = load(case.name)
        for k in range(len(case.pairs)):
            out = bufs[k][1].cpu().numpy().view(oracle.NP[case.dtype])
            if not matches(fx, f"C{k}_r0", out):
                bad.append(f"{case.name} C{k}")
    m = 12288  # a 1.2 GB package: one unchunked RCCL self send/recv of it loses half
    A = torch.rand(m * m, dtype=torch.float64, device="cuda")
    Cm = torch.zeros(m * m, dtype=torch.float64, device="cuda")
    LA = costa.block_cyclic_layout(m, m, 256, 256, 1, 1, m, m, 1, 1, "R", 0, 0, A.data_ptr(), m, "C", 0)
    LC = costa.block_cyclic_layout(m, m, 256, 256, 1, 1, m, m, 1, 1, "R", 0, 0, Cm.data_ptr(), m, "C", 0)
    costa.transform(LA, LC, comm, "T", 1.0, 0.0)
    torch.cuda.synchronize()
    if not torch.equal(Cm.view(m, m), A.view(m, m).t()):
        bad.append(f"{m}^2 fp64 T")
    # alpha, beta through several exchange rounds (a 300 MB package: 4 rounds) with 80^2 blocks,
    # ragged at the edge, whose tiles merge inside each round's pack and unpack lists
    m2 = 6144
    rng2 = np.random.default_rng(11)
    a2 = rng2.standard_normal(m2 * m2)
    c2 = rng2.standard_normal(m2 * m2)
    A2, C2 = torch.from_numpy(a2).cuda(), torch.from_numpy(c2).cuda()
    LA2 = costa.block_cyclic_layout(m2, m2, 80, 80, 1, 1, m2, m2, 1, 1, "R", 0, 0, A2.data_ptr(), m2, "C", 0)
    LC2 = costa.block_cyclic_layout(m2, m2, 80, 80, 1, 1, m2, m2, 1, 1, "R", 0, 0, C2.data_ptr(), m2, "C", 0)
    costa.transform(LA2, LC2, comm, "T", -0.75, 1.5)
    exp2 = 1.5 * c2 + -0.75 * a2.reshape(m2, m2).T.copy().reshape(-1)
    if not np.array_equal(C2.cpu().numpy().view(np.uint64), exp2.view(np.uint64)):
        bad.append(f"{m2}^2 fp64 T alpha beta 80^2 blocks")
    del A2, C2
    # ragged custom layouts whose C blocks are their own buffers (test_gpu_cblock's geometry): the
    # unpack lists' destination-block groups, 'N' and 'T' alpha / beta, against the oracle
    from casegen import Custom
    rng3 = np.random.default_rng(23)

    def splits(n, lo, hi):
        sp = [0]
        while sp[-1] < n:
            sp.append(min(n, sp[-1] + int(rng3.integers(lo, hi + 1))))
        return sp
    for op3, al3, be3 in (("N", 1.0, 0.0), ("T", -0.5, 2.0)):
        m3, n3 = 1100, 900
        am, an = (n3, m3) if op3 == "T" else (m3, n3)
        rs, cs = splits(am, 8, 60), splits(an, 8, 60)
        CA = Custom(rs, cs, np.zeros((len(rs) - 1, len(cs) - 1), np.int32), gap=1)
        rs, cs = splits(m3, 30, 220), splits(n3, 30, 220)
        CC = Custom(rs, cs, np.zeros((len(rs) - 1, len(cs) - 1), np.int32), gap=0)
        a3 = oracle.gen(oracle.FLOAT, 1, 0, CA.buf_elems(0, 1))
        c3 = oracle.gen(oracle.FLOAT, 2, 0, CC.buf_elems(0, 1))
        exp3 = c3.copy()
        oracle.transform(oracle.FLOAT, op3, al3, be3, CA.geom(1), [a3], CC.geom(1), [exp3])
        da3, dc3 = dev(a3), dev(c3)
        costa.transform(CA.make_layout(0, da3.data_ptr(), 1, oracle.FLOAT),
                        CC.make_layout(0, dc3.data_ptr(), 1, oracle.FLOAT), comm, op3, al3, be3)
        torch.cuda.synchronize()
        if dc3.cpu().numpy().tobytes() != exp3.tobytes():
            bad.append(f"custom {op3} groups")
    # stream-ordered: A changes on torch's stream between queued transforms
    s = torch.cuda.current_stream()
    for k in range(4):
        A.mul_(-1.5)
        costa.transform_async(LA, LC, comm, "T", 1.0, 0.0, stream=s)
    costa.synchronize(comm)
    torch.cuda.synchronize()
    if not torch.equal(Cm.view(m, m), A.view(m, m).t()):
        bad.append(f"{m}^2 fp64 T async")
    # host-resident layouts (the ScaLAPACK situation): the pipelined staging gathers the pack
    # groups into the send buffer, exchanges with itself over RCCL and brings the unpack groups
    # back to host memory; the mirror scheme (mode 0) as a cross-check
    host_groups = 0
    direct_groups = 0
    for hmode in (1, 0, "pinned"):
        costa.set_host_staging(1 if hmode == "pinned" else hmode)
        g0 = costa.get_stats()["host_groups"]
        d0 = costa.get_stats()["host_direct_groups"]
        keep = []
        for case in all_cases():
            if case.P != 1:
                continue
            bufs = [case.inputs(k, 0) for k in range(len(case.pairs))]
            if hmode == "pinned":  # page-locked caller memory: groups move by strided DMA
                bufs = [tuple(pinned(x, keep) for x in b) for b in bufs]
            As = [case.layout_A(k, 0, bufs[k][0].ctypes.data) for k in range(len(case.pairs))]
            Cs = [case.layout_C(k, 0, bufs[k][1].ctypes.data) for k in range(len(case.pairs))]
            eff = [case.effective(k) for k in range(len(case.pairs))]
            costa.transform_batch(As, Cs, comm, [e[0] for e in eff], [e[1] for e in eff],
                                  [e[2] for e in eff])
            fx = load(case.name)
            for k in range(len(case.pairs)):
                if not matches(fx, f"C{k}_r0", bufs[k][1]):
                    bad.append(f"host mode {hmode} {case.name} C{k}")
        hm, hn = 3000, 2500  # many groups, ops cut over a slot when COSTA_HOST_SLOT_MIB is small
        rng = np.random.default_rng(3)
        ha = rng.standard_normal(hm * hn)
        c0 = rng.standard_normal(hn * hm)
        hc = c0.copy()
        if hmode == "pinned":
            ha, hc = pinned(ha, keep), pinned(hc, keep)
        HA = costa.block_cyclic_layout(hm, hn, 512, 384, 1, 1, hm, hn, 1, 1, "R", 0, 0, ha, hm, "C", 0)
        HC = costa.block_cyclic_layout(hn, hm, 384, 512, 1, 1, hn, hm, 1, 1, "R", 0, 0, hc, hn, "C", 0)
        costa.transform(HA, HC, comm, "T", -0.75, 1.5)
        exp = 1.5 * c0 + -0.75 * ha.reshape(hn, hm).T.copy().reshape(-1)
        if not np.array_equal(hc.view(np.uint64), exp.view(np.uint64)):
            bad.append(f"host mode {hmode} {hm}x{hn} T axpby")
        groups = costa.get_stats()["host_groups"] - g0
        if (groups > 0) != (hmode != 0):
            bad.append(f"host mode {hmode}: {groups} pipeline groups")
        host_groups += groups
        if hmode == "pinned":
            direct_groups = costa.get_stats()["host_direct_groups"] - d0
        del keep
    costa.set_host_staging(1)
    print("HOST", host_groups)
    print("DIRECT", direct_groups)
    st = costa.get_stats()
    print("LISTS", st["device_lists"])  # work lists whose groups the GPU built
    for b in bad:
        print("FAIL", b)
    print("OK" if not bad else "BAD", n + 1, st["pack_launches"], st["unpack_launches"],
          st["local_launches"])
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
