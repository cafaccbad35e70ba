"""GPU parity: the HIP kernels (through the C ABI) against the reference's golden vectors and
the CPU oracle.  Bit-exact for every case (copies and fp arithmetic alike: contraction is off
on both sides); the fp tolerance is therefore 0 ulp.

Multi-rank golden cases run on ONE GPU: each rank's plan is executed by the real kernels
(pack / local / unpack launches via costa_hip_execute_tiles) and the exchange is emulated with
device-to-device copies of exactly the segments ncclSend/ncclRecv would move.  The RCCL path
itself runs in bench.py on multi-GPU nodes.
"""
import hashlib

import numpy as np
import pytest

import oracle
from cases import BC, Case, Pair, all_cases, special_cases
from golden_io import first_mismatch, load, matches

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def dev(arr: np.ndarray):
    """device copy of a numpy buffer (raw bytes, any dtype)"""
    return torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8).copy()).cuda()


def host(t, dtype) -> np.ndarray:
    return t.cpu().numpy().view(dtype)


@pytest.fixture(scope="module")
def gpu(costa):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return costa


# ------------------------------------------------------------------ known answers
IN8x4 = np.array([9, 1, 1, -1, 7, 3, 4, -1, 5, 5, 1, -1, 9, 2, 3, -1,
                  7, 6, 5, -1, 2, 2, 4, -1, 3, 7, 4, -1, 3, 8, 1, -1], np.int32)


@pytest.mark.parametrize("name,args,size", [
    ("copy2D_row_major_out", (8, 3, 4, False, 5, False), 40),
    ("copy2D_col_major_out", (3, 8, 4, True, 5, True), 40),
    ("row_to_col_major_out", (8, 3, 4, False, 10, True), 30),
])
def test_kat_small(gpu, name, args, size):
    nr, nc, ls, scm, ld, dcm = args
    src = dev(IN8x4)
    dst = dev(np.zeros(size, np.int32))
    gpu.copy_and_transform(gpu.INT32, nr, nc, src.data_ptr(), ls, scm, dst.data_ptr(), ld, dcm)
    torch.cuda.synchronize()
    assert (host(dst, np.int32) == load("kat")[name]).all()


def test_kat_col_to_row_major(gpu):
    from test_oracle_golden import kat_inputs_col_to_row
    inp = kat_inputs_col_to_row()
    src = dev(inp)
    dst = dev(np.zeros(1000 * 501, np.int32))
    gpu.copy_and_transform(gpu.INT32, 1000, 500, src.data_ptr(), 1100, True, dst.data_ptr(), 501,
                           False)
    out = host(dst, np.int32)
    assert (out.reshape(1000, 501)[:, :500] == inp.reshape(500, 1100)[:, :1000].T).all()
    assert hashlib.sha256(out.tobytes()).digest() == bytes(load("kat")["sha_col_to_row_major_out"])


# ------------------------------------------------------------------ golden cases
def _run_single_rank(costa, case, on_device=True):
    bufs = [case.inputs(k, 0) for k in range(len(case.pairs))]
    dbufs = [(dev(a), dev(c)) for a, c in bufs] if on_device else bufs
    As, Cs = [], []
    for k, p in enumerate(case.pairs):
        a, c = dbufs[k]
        pa = a.data_ptr() if on_device else a.ctypes.data
        pc = c.data_ptr() if on_device else c.ctypes.data
        As.append(case.layout_A(k, 0, pa))
        Cs.append(case.layout_C(k, 0, pc))
    eff = [case.effective(k) for k in range(len(case.pairs))]
    comm = costa.Comm.self(0)
    costa.transform_batch(As, Cs, comm, [e[0] for e in eff], [e[1] for e in eff],
                          [e[2] for e in eff])
    out = []
    for k in range(len(case.pairs)):
        c = dbufs[k][1]
        out.append(host(c, oracle.NP[case.dtype]) if on_device else c)
    return out


def _run_emulated_ranks(costa, case):
    P, dt = case.P, oracle.NP[case.dtype]
    bufs = [[tuple(dev(x) for x in case.inputs(k, r)) for k in range(len(case.pairs))]
            for r in range(P)]
    eff = [case.effective(k) for k in range(len(case.pairs))]
    plans, keep = [], []
    for r in range(P):
        As = [case.layout_A(k, r, bufs[r][k][0].data_ptr()) for k in range(len(case.pairs))]
        Cs = [case.layout_C(k, r, bufs[r][k][1].data_ptr()) for k in range(len(case.pairs))]
        keep.append((As, Cs))
        plans.append(costa.plan_export(As, Cs, r, P, [e[0] for e in eff], [e[1] for e in eff],
                                       [e[2] for e in eff]))
    E = np.dtype(dt).itemsize
    send = [torch.zeros(max(1, p.send_elems) * E, dtype=torch.uint8, device="cuda") for p in plans]
    recv = [torch.zeros(max(1, p.recv_elems) * E, dtype=torch.uint8, device="cuda") for p in plans]
    for r, p in enumerate(plans):
        if p.pack_ops.size:
            costa.execute_tiles(case.dtype, p.pack_ops, p.scalars, 0, send[r].data_ptr())
    for r in range(P):
        for q in range(P):
            n = int(plans[r].recv_counts[q]) * E
            d, s = int(plans[r].recv_displs[q]) * E, int(plans[q].send_displs[r]) * E
            if n:
                recv[r][d:d + n].copy_(send[q][s:s + n])
    torch.cuda.synchronize()
    for r, p in enumerate(plans):
        if p.unpack_ops.size:
            costa.execute_tiles(case.dtype, p.unpack_ops, p.scalars, recv[r].data_ptr(), 0)
        if p.local_ops.size:
            costa.execute_tiles(case.dtype, p.local_ops, p.scalars, 0, 0)
    return [[host(bufs[r][k][1], dt) for k in range(len(case.pairs))] for r in range(P)]


@pytest.mark.parametrize("case", all_cases(), ids=lambda c: c.name)
def test_golden_on_gpu(gpu, case):
    fx = load(case.name)
    if case.P == 1:
        got = [_run_single_rank(gpu, case)]
    else:
        got = _run_emulated_ranks(gpu, case)
    for r in range(case.P):
        for k in range(len(case.pairs)):
            key = f"C{k}_r{r}"
            assert matches(fx, key, got[r][k]), f"{case.name} {key}: " + first_mismatch(
                fx, key, got[r][k])


@pytest.mark.parametrize("case", [c for c in all_cases() if c.P == 1][:8], ids=lambda c: c.name)
def test_golden_host_staged(gpu, case):
    """host-resident matrices (the reference's own situation): staged through HBM"""
    fx = load(case.name)
    got = _run_single_rank(gpu, case, on_device=False)
    for k in range(len(case.pairs)):
        assert matches(fx, f"C{k}_r0", got[k])


@pytest.mark.parametrize("ld_pad,sub,beta", [(0, False, 0.0), (3, False, 0.0), (0, True, 0.0),
                                             (0, False, 0.5)])
def test_host_staged_c_upload_rules(gpu, ld_pad, sub, beta):
    """The staged path skips uploading C ranges the kernels overwrite completely (beta = 0, no
    ld padding, whole matrix).  Padding bytes, rows outside a sub-matrix and beta != 0 must
    still see the caller's C: the whole host buffer is compared, padding included."""
    m, n, b = 300, 200, 64
    rng = np.random.default_rng(7)
    a = rng.standard_normal(m * n)                     # A: m x n, col-major, ld m
    ldc = n + ld_pad
    c0 = rng.standard_normal(ldc * m)                  # C: n x m, col-major, ld n + pad
    c = c0.copy()
    sm, sn = (m - 40, n - 30) if sub else (m, n)       # sub(C) = op(sub(A)): sn x sm
    LA = gpu.block_cyclic_layout(m, n, b, b, 1, 1, sm, sn, 1, 1, "R", 0, 0, a, m, "C", 0)
    LC = gpu.block_cyclic_layout(n, m, b, b, 1, 1, sn, sm, 1, 1, "R", 0, 0, c, ldc, "C", 0)
    gpu.transform(LA, LC, gpu.Comm.self(0), "T", 1.5, beta)
    exp = c0.copy().reshape(m, ldc)                    # row j of exp = column j of C
    at = a.reshape(n, m)[:sn, :sm]                     # at[j, i] = A(i, j) = op(A)(j, i)
    cur = exp[:sm, :sn]
    new = 1.5 * at.T if beta == 0 else beta * cur + 1.5 * at.T
    exp[:sm, :sn] = new
    assert np.array_equal(c.view(np.uint64), exp.reshape(-1).view(np.uint64))


# ------------------------------------------------------------------ edge cases vs oracle
def assert_bits_equal_or_both_nan(got, expected):
    """Bit-exact, except NaNs GENERATED by arithmetic (inf*0, inf-inf): x86 produces the
    'default NaN' with the sign bit set (0xffc00000), the GPU 0x7fc00000; the sign/payload
    of a generated NaN is platform-defined, so both-NaN counts as equal.  Non-NaN results,
    infinities, signed zeros and denormals must match bit for bit."""
    g = got.view(np.float32 if got.dtype in (np.float32, np.complex64) else np.float64)
    e = expected.view(g.dtype)
    same = (g.view(np.uint8).reshape(g.size, -1) == e.view(np.uint8).reshape(e.size, -1)).all(1)
    ok = same | (np.isnan(g) & np.isnan(e))
    assert ok.all(), f"{(~ok).sum()} elements differ; first {np.nonzero(~ok)[0][:5]}"


SPECIAL = np.array([0.0, -0.0, 1.0, -1.0, 1e-310, -1e-310, 1e308, -1e308, 3.5, -2.25, np.inf,
                    -np.inf, np.nan], np.float64)


@pytest.mark.parametrize("case", special_cases(), ids=lambda c: c.name)
def test_special_values_golden(gpu, case):
    """inf / NaN / signed zeros / huge values against the REFERENCE's own outputs: the complex
    products recover infinities as GCC's __muldc3 / __mulsc3 do (C99 Annex G), e.g.
    (inf + inf i)(1 + 0i) = inf + inf i; generated NaNs may differ in sign only"""
    fx = load(case.name)
    got = [_run_single_rank(gpu, case)] if case.P == 1 else _run_emulated_ranks(gpu, case)
    for r in range(case.P):
        for k in range(len(case.pairs)):
            assert_bits_equal_or_both_nan(got[r][k], fx[f"C{k}_r{r}"])


@pytest.mark.parametrize("dtype", [0, 1, 2, 3])
@pytest.mark.parametrize("trans", ["N", "T", "C"])
@pytest.mark.parametrize("ab", [(1, 0), (0, 0), (0.5, 0), (1, 1), (-1.5, 0.25)])
@pytest.mark.parametrize("ords", [("C", "C"), ("R", "C"), ("C", "R")])
def test_special_values_vs_oracle(gpu, dtype, trans, ab, ords):
    """signed zeros, denormals, huge values; the complex alpha = 1 'copy' fast path vs the
    transposing path (signed-zero sensitive); beta = 0 must not read C (C holds NaN)."""
    m, n = 37, 29
    rng = np.random.default_rng(7)
    a_case = BC(n if trans != "N" else m, m if trans != "N" else n, 8, 5, ord=ords[0])
    c_case = BC(m, n, 6, 7, ord=ords[1])
    npd = oracle.NP[dtype]
    na, nc = a_case.buf_elems(0, 1), c_case.buf_elems(0, 1)
    if dtype in (2, 3):
        a = (rng.choice(SPECIAL, na) + 1j * rng.choice(SPECIAL, na)).astype(npd)
    else:
        a = rng.choice(SPECIAL, na).astype(npd)
    beta = ab[1]
    c = np.full(nc, np.nan, npd) if beta == 0 else rng.choice(SPECIAL, nc).astype(npd)
    alpha = ab[0] if dtype < 2 else complex(ab[0], 0.5 if ab[0] not in (0, 1) else 0)
    expected = c.copy()
    oracle.transform(dtype, trans, alpha, beta, a_case.geom(1), [a], c_case.geom(1), [expected])
    da, dc = dev(a), dev(c)
    A = a_case.make_layout(0, da.data_ptr(), 1, dtype)
    Cl = c_case.make_layout(0, dc.data_ptr(), 1, dtype)
    gpu.transform(A, Cl, gpu.Comm.self(0), trans, alpha, beta)
    got = host(dc, npd)
    # C was pre-filled with NaN when beta == 0: any read of C would leave NaN where the
    # oracle (which never reads C then) has a number
    assert_bits_equal_or_both_nan(got, expected)


# ------------------------------------------------------------------ full-size properties
def test_cfg2_full_size_transpose(gpu):
    """BASELINE cfg 2 at full size: pxtran fp64 16384^2, 256^2 blocks, alpha=1, beta=0.
    Property: C == A^T exactly (bit copy through alpha*x with alpha = 1)."""
    n, b = 16384, 256
    A = torch.randn(n, n, dtype=torch.float64, device="cuda")
    Cm = torch.full((n, n), float("nan"), dtype=torch.float64, device="cuda")
    # column-major local storage: element (i, j) at i + j*n  ==  tensor[j, i]
    LA = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), n, "C", 0)
    LC = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, Cm.data_ptr(), n, "C", 0)
    gpu.transform(LA, LC, gpu.Comm.self(0), "T", 1.0, 0.0)
    torch.cuda.synchronize()
    assert torch.equal(Cm, A.t())


def test_full_size_axpby_checksum(gpu):
    """8192^2 fp64 'T' with alpha, beta != 0 against numpy's separately rounded
    beta*C + alpha*A^T (no fma), compared bit for bit."""
    n, b = 8192, 256
    rng = np.random.default_rng(11)
    a = rng.standard_normal(n * n)
    c = rng.standard_normal(n * n)
    alpha, beta = 0.75, -1.25
    expected = (beta * c.reshape(n, n)) + (alpha * a.reshape(n, n).T)
    da, dc = dev(a), dev(c)
    LA = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, da.data_ptr(), n, "C", 0)
    LC = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, dc.data_ptr(), n, "C", 0)
    gpu.transform(LA, LC, gpu.Comm.self(0), "T", alpha, beta)
    got = host(dc, np.float64).reshape(n, n)
    assert got.tobytes() == np.ascontiguousarray(expected).tobytes()


def test_async_stream_ordered(gpu):
    """stream-ordered transforms: queued back to back with changing scalars on the same
    handles, consumed by torch on the same stream without a host sync"""
    n, b = 1024, 128
    A = torch.arange(n * n, dtype=torch.float64, device="cuda") % 97 - 48
    Cm = torch.full((n * n,), float("nan"), dtype=torch.float64, device="cuda")
    LA = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), n, "C", 0)
    LC = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, Cm.data_ptr(), n, "C", 0)
    comm = gpu.Comm.self(0)
    s = torch.cuda.current_stream()
    gpu.transform_async(LA, LC, comm, "T", 2.0, 0.0, stream=s)   # C = 2 A^T   (C = NaN not read)
    gpu.transform_async(LA, LC, comm, "T", 3.0, 1.0, stream=s)   # C = C + 3 A^T = 5 A^T
    gpu.transform_async(LA, LC, comm, "T", -1.0, 0.5, stream=s)  # C = C/2 - A^T = 1.5 A^T
    got = Cm.view(n, n).clone()  # queued on s after the transforms
    assert torch.equal(got, 1.5 * A.view(n, n).t())


def test_async_rejects_host_layouts(gpu):
    a = np.zeros(64 * 64)
    c = np.zeros(64 * 64)
    LA = gpu.block_cyclic_layout(64, 64, 32, 32, 1, 1, 64, 64, 1, 1, "R", 0, 0, a, 64, "C", 0)
    LC = gpu.block_cyclic_layout(64, 64, 32, 32, 1, 1, 64, 64, 1, 1, "R", 0, 0, c, 64, "C", 0)
    with pytest.raises(gpu.CostaError, match="device-resident"):
        gpu.transform_async(LA, LC, gpu.Comm.self(0), "T", 1.0, 0.0)


def test_plan_cache_reuse(gpu):
    """the second identical call hits the plan cache and gives the same result"""
    case = [c for c in all_cases() if c.name == "block_cyclic"][0]
    gpu.get_stats(reset=True)
    r1 = _run_single_rank(gpu, case)
    r2 = _run_single_rank(gpu, case)
    assert r1[0].tobytes() == r2[0].tobytes()
    s = gpu.get_stats()
    assert s["transforms"] == 2


@pytest.mark.parametrize("dtype,lda,ldc", [(1, 16385, 16385), (1, 16384, 16387), (0, 16386, 16385),
                                           (0, 16387, 16386), (4, 16385, 16387)],
                         ids=["f64-odd", "f64-dst-odd", "f32-2-1", "f32-3-2", "i32-1-3"])
def test_unaligned_lld_full_size(gpu, dtype, lda, ldc):
    """a ScaLAPACK-sized 'T' with leading dimensions off the 16-byte grid (lld = LOCr + pad):
    the large shape re-cuts its stores into aligned chunks across lanes (store_shifted);
    C == A^T bit for bit, padding rows untouched"""
    n, b = 16384, 256
    tdt = {0: torch.float32, 1: torch.float64, 4: torch.int32}[dtype]
    if tdt == torch.int32:
        A = torch.randint(-2**31, 2**31 - 1, (n, lda), dtype=torch.int32, device="cuda")
    else:
        A = torch.randn(n, lda, dtype=tdt, device="cuda")
    Cm = torch.full((n, ldc), 7, dtype=tdt, device="cuda")
    LA = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), lda, "C", 0,
                                 dtype=dtype)
    LC = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, Cm.data_ptr(), ldc, "C", 0,
                                 dtype=dtype)
    gpu.transform(LA, LC, gpu.Comm.self(0), "T", 1, 0)
    torch.cuda.synchronize()
    assert torch.equal(Cm[:, :n], A[:, :n].t())
    assert bool((Cm[:, n:] == 7).all())


@pytest.mark.parametrize("dtype", [0, 1, 4])
@pytest.mark.parametrize("pad", [1, 2, 3])
@pytest.mark.parametrize("ab", [(1, 0), (0, 0), (0.5, 0), (-1.5, 0.25)])
@pytest.mark.parametrize("geo", [(1500, 1100, 256, 256, 1, 1), (1437, 1203, 300, 170, 5, 9),
                                 (4100, 700, 1024, 700, 3, 1)],
                         ids=["b256", "ragged-sub", "tall"])
def test_unaligned_skew_vs_oracle(gpu, dtype, pad, ab, geo):
    """'T' into destination columns off the 16-byte grid (lld = LOCr + pad): the skew shape
    (granule-cut sub-tiles) including ops that read C (beta != 0), sub-matrices that start
    inside a granule, op lengths that are no multiple of the sub-tile; bit-exact vs the oracle,
    padding rows untouched"""
    m, n, mb, nb, ia, ja = geo
    rng = np.random.default_rng(17 + pad)
    a_case = BC(n + ja, m + ia, nb, mb, ia=ja, ja=ia, subm=n, subn=m, lld_pad=pad)
    c_case = BC(m + ia, n + ja, mb, nb, ia=ia, ja=ja, subm=m, subn=n, lld_pad=pad + 1)
    npd = oracle.NP[dtype]
    na, nc = a_case.buf_elems(0, 1), c_case.buf_elems(0, 1)
    if dtype == 4:
        a = rng.integers(-2**20, 2**20, na).astype(npd)  # products stay inside int32
        c = rng.integers(-2**20, 2**20, nc).astype(npd)
        alpha, beta = int(ab[0] * 2), int(ab[1] * 4)
    else:
        a = rng.standard_normal(na).astype(npd)
        c = rng.standard_normal(nc).astype(npd)
        alpha, beta = ab
    expected = c.copy()
    oracle.transform(dtype, "T", alpha, beta, a_case.geom(1), [a], c_case.geom(1), [expected])
    da, dc = dev(a), dev(c)
    A = a_case.make_layout(0, da.data_ptr(), 1, dtype)
    Cl = c_case.make_layout(0, dc.data_ptr(), 1, dtype)
    gpu.transform(A, Cl, gpu.Comm.self(0), "T", alpha, beta)
    got = host(dc, npd)
    assert got.tobytes() == expected.tobytes()


@pytest.mark.parametrize("dtype", [0, 1, 4])
@pytest.mark.parametrize("pads", [(0, 1), (0, 2), (0, 3), (1, 2), (3, 1)], ids=lambda p: f"a{p[0]}c{p[1]}")
@pytest.mark.parametrize("ab", [(1, 0), (-1.5, 0.25)], ids=["copy", "axpby"])
@pytest.mark.parametrize("geo", [(1500, 1100, 256, 256, 1, 1), (1437, 1203, 300, 170, 5, 9)],
                         ids=["b256", "ragged-sub"])
def test_unaligned_copy_vs_oracle(gpu, dtype, pads, ab, geo):
    """'N' (p?gemr2d) into destination columns off the 64-byte grid (lld = LOCr + pad, sub-matrices
    starting inside a granule): the copies cut at each column's granules (engine.cpp
    granule_split) where that is on, the large copy shape otherwise; beta != 0 cases read C;
    bit-exact vs the oracle over the whole buffer, padding rows untouched"""
    m, n, mb, nb, ia, ja = geo
    pa, pc = pads
    rng = np.random.default_rng(41 + pa + 7 * pc)
    a_case = BC(m + ia, n + ja, mb, nb, ia=ia, ja=ja, subm=m, subn=n, lld_pad=pa)
    c_case = BC(m + ia, n + ja, mb, nb, ia=ia, ja=ja, subm=m, subn=n, lld_pad=pc)
    npd = oracle.NP[dtype]
    na, nc = a_case.buf_elems(0, 1), c_case.buf_elems(0, 1)
    if dtype == 4:
        a = rng.integers(-2**20, 2**20, na).astype(npd)
        c = rng.integers(-2**20, 2**20, nc).astype(npd)
        alpha, beta = int(ab[0] * 2), int(ab[1] * 4)
    else:
        a = rng.standard_normal(na).astype(npd)
        c = rng.standard_normal(nc).astype(npd)
        alpha, beta = ab
    expected = c.copy()
    oracle.transform(dtype, "N", alpha, beta, a_case.geom(1), [a], c_case.geom(1), [expected])
    da, dc = dev(a), dev(c)
    A = a_case.make_layout(0, da.data_ptr(), 1, dtype)
    Cl = c_case.make_layout(0, dc.data_ptr(), 1, dtype)
    gpu.transform(A, Cl, gpu.Comm.self(0), "N", alpha, beta)
    got = host(dc, npd)
    assert got.tobytes() == expected.tobytes()


@pytest.mark.parametrize("dtype,lda,ldc", [(1, 16384, 16386), (1, 16385, 16385), (0, 16384, 16388),
                                           (4, 16384, 16387)],
                         ids=["f64-c2", "f64-odd", "f32-c4", "i32-c3"])
def test_unaligned_copy_full_size(gpu, dtype, lda, ldc):
    """a ScaLAPACK-sized p?gemr2d copy into columns off the 64-byte grid: C == A bit for bit,
    padding rows untouched"""
    n, b = 16384, 256
    tdt = {0: torch.float32, 1: torch.float64, 4: torch.int32}[dtype]
    if tdt == torch.int32:
        A = torch.randint(-2**31, 2**31 - 1, (n, lda), dtype=torch.int32, device="cuda")
    else:
        A = torch.randn(n, lda, dtype=tdt, device="cuda")
    Cm = torch.full((n, ldc), 7, dtype=tdt, device="cuda")
    LA = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, A.data_ptr(), lda, "C", 0,
                                 dtype=dtype)
    LC = gpu.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, Cm.data_ptr(), ldc, "C", 0,
                                 dtype=dtype)
    gpu.transform(LA, LC, gpu.Comm.self(0), "N", 1, 0)
    torch.cuda.synchronize()
    assert torch.equal(Cm[:, :n], A[:, :n])
    assert bool((Cm[:, n:] == 7).all())


@pytest.mark.parametrize("dtype", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("trans", ["N", "T", "C"])
@pytest.mark.parametrize("geo", [(1000, 1100, 24, 24, 1, 1, 0), (1037, 997, 24, 20, 3, 5, 2),
                                 (2048, 700, 16, 16, 1, 1, 1)],
                         ids=["b24", "ragged-sub-pad", "b16-pad"])
def test_merged_small_blocks_vs_oracle(gpu, dtype, trans, geo):
    """small blocks on one rank: the tiles of the local matrix continue each other on both sides
    and merge into large-shape ops (engine.cpp merge_filled); ragged last blocks, sub-matrices
    and ld padding (16-byte alignment of the merged op from its first tile only); alpha, beta !=
    0 on half the cases; bit-exact vs the oracle"""
    if trans == "C" and dtype not in (2, 3):
        pytest.skip("conjugate: complex types only")
    m, n, mb, nb, ia, ja, pad = geo
    rng = np.random.default_rng(29 + mb + pad)
    tr = trans != "N"
    if tr:
        a_case = BC(n + ja, m + ia, nb, mb, ia=ja, ja=ia, subm=n, subn=m, lld_pad=pad)
    else:
        a_case = BC(m + ia, n + ja, mb, nb, ia=ia, ja=ja, subm=m, subn=n, lld_pad=pad)
    c_case = BC(m + ia, n + ja, mb, nb, ia=ia, ja=ja, subm=m, subn=n, lld_pad=pad)
    npd = oracle.NP[dtype]
    na, nc = a_case.buf_elems(0, 1), c_case.buf_elems(0, 1)
    axpby = (m + dtype) % 2 == 0
    if dtype == 4:
        a = rng.integers(-2**20, 2**20, na).astype(npd)
        c = rng.integers(-2**20, 2**20, nc).astype(npd)
        alpha, beta = (3, -2) if axpby else (1, 0)
    else:
        a = oracle.gen(dtype, 3, 0, na)
        c = oracle.gen(dtype, 4, 0, nc)
        alpha, beta = ((0.75 - 0.5j, 1.25 + 0.25j) if dtype in (2, 3) else (-1.5, 0.25)) if axpby else (1, 0)
    expected = c.copy()
    oracle.transform(dtype, trans, alpha, beta, a_case.geom(1), [a], c_case.geom(1), [expected])
    da, dc = dev(a), dev(c)
    A = a_case.make_layout(0, da.data_ptr(), 1, dtype)
    Cl = c_case.make_layout(0, dc.data_ptr(), 1, dtype)
    gpu.transform(A, Cl, gpu.Comm.self(0), trans, alpha, beta)
    got = host(dc, npd)
    assert got.tobytes() == expected.tobytes()
