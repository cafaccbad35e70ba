"""GPU: host-resident layouts (the reference's own situation: the path starts and ends in each
rank's host buffers) through both host staging modes of engine.cpp / host_pipe.cpp:
  1  pipelined: local tiles in groups through pinned/device slot rings (gather -> H2D ->
     kernels -> D2H -> scatter), several groups in flight
  0  mirror: every spanned byte range up, kernels, target ranges down
Both must match the reference bit for bit (0 ulp: contraction is off), leave every
byte of C the transform does not write untouched, and mode 1 must actually run the pipeline
(costa_stats_t::host_groups)."""
import json
import os

import numpy as np
import pytest

import oracle
from casegen import BC
from cases import all_cases
from golden_io import first_mismatch, load, matches
from test_gpu_parity import _run_single_rank

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(costa):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return costa


def _with_mode(costa, mode, fn):
    costa.set_host_staging(mode)
    try:
        costa.get_stats(reset=True)
        out = fn()
        return out, costa.get_stats(reset=True)
    finally:
        costa.set_host_staging(1)


SINGLE = [c for c in all_cases() if c.P == 1]
_DX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "host_direct.json")
DIRECT_EXPECTED = json.load(open(_DX)) if os.path.exists(_DX) else {}


@pytest.mark.parametrize("mode", [1, 0])
@pytest.mark.parametrize("case", SINGLE, ids=lambda c: c.name)
def test_golden_host_resident(gpu, case, mode):
    got, st = _with_mode(gpu, mode, lambda: _run_single_rank(gpu, case, on_device=False))
    fx = load(case.name)
    for k in range(len(case.pairs)):
        key = f"C{k}_r0"
        assert matches(fx, key, got[k]), f"{case.name} {key}: " + first_mismatch(fx, key, got[k])
    if mode == 0:
        assert st["host_groups"] == 0
    elif len(case.pairs) == 1 and np.prod(case.pairs[0].C.shape()) > 0:
        assert st["host_groups"] >= 1, "pipelined staging did not run"


# (m, n, mb, nb): many tiles over several 64 MiB groups; one 96 MB block cut into pieces;
# ragged small blocks in one group
SHAPES = [(6000, 5000, 1000, 700), (4000, 3000, 4000, 3000), (1000, 900, 100, 70)]


@pytest.mark.parametrize("mode", [1, 0])
@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("trans,alpha,beta", [("T", 1.0, 0.0), ("N", 1.0, 0.0), ("T", -0.75, 1.5),
                                              ("N", 2.0, 0.5)])
def test_large_host_vs_numpy(gpu, mode, shape, trans, alpha, beta):
    m, n, mb, nb = shape
    rng = np.random.default_rng(11)
    a = rng.standard_normal(m * n)                        # A: m x n col-major, ld m
    cm, cn = (n, m) if trans == "T" else (m, n)           # C = op(A) shape, col-major, ld cm
    c0 = rng.standard_normal(cm * cn)
    c = c0.copy()
    LA = gpu.block_cyclic_layout(m, n, mb, nb, 1, 1, m, n, 1, 1, "R", 0, 0, a, m, "C", 0)
    cmb, cnb = (nb, mb) if trans == "T" else (mb, nb)
    LC = gpu.block_cyclic_layout(cm, cn, cmb, cnb, 1, 1, cm, cn, 1, 1, "R", 0, 0, c, cm, "C", 0)
    _, st = _with_mode(gpu, mode, lambda: gpu.transform(LA, LC, gpu.Comm.self(0), trans, alpha,
                                                        beta))
    # 'T': C(j, i) = A(i, j) sits at c[j + i*n]; as an (m, n) array that is A's (n, m) view
    # transposed
    x = a.reshape(n, m).T.copy().reshape(-1) if trans == "T" else a
    exp = alpha * x if beta == 0 else beta * c0 + alpha * x
    assert np.array_equal(c.view(np.uint64), exp.view(np.uint64))
    if mode == 1:
        assert st["host_groups"] >= (2 if m * n * 8 > (64 << 20) else 1)


@pytest.mark.parametrize("mode", [1, 0])
def test_complex_conj_orderings_host_vs_oracle(gpu, mode):
    """c128 'C' (conjugate transpose) with alpha, beta != 0, source row-major and target
    column-major (an ordering mismatch is itself a transpose), ld padding on both sides and a
    sub-matrix: the padding and the rows outside sub(C) must come back unchanged."""
    dt = oracle.CDOUBLE
    m, n = 2000, 1500
    a_case = BC(n + 7, m + 5, 300, 200, ia=4, ja=3, subm=n, subn=m, ord="R", lld_pad=9)
    c_case = BC(m + 3, n + 2, 256, 160, ia=2, ja=1, subm=m, subn=n, ord="C", lld_pad=5)
    a = oracle.gen(dt, 1, 0, a_case.buf_elems(0, 1))
    c = oracle.gen(dt, 2, 0, c_case.buf_elems(0, 1))
    alpha, beta = 0.75 - 0.5j, 1.25 + 0.25j
    expected = c.copy()
    oracle.transform(dt, "C", alpha, beta, a_case.geom(1), [a], c_case.geom(1), [expected])
    A = a_case.make_layout(0, a.ctypes.data, 1, dt)
    C = c_case.make_layout(0, c.ctypes.data, 1, dt)
    _, st = _with_mode(gpu, mode, lambda: gpu.transform(A, C, gpu.Comm.self(0), "C", alpha, beta))
    assert c.tobytes() == expected.tobytes()
    assert (st["host_groups"] >= 1) == (mode == 1)


def test_pipeline_repeated_calls_and_mode_switch(gpu):
    """the same host layouts called repeatedly (plan cache hits, ring reuse), switching modes
    in between: every call's result is exact"""
    m, n, b = 4096, 3072, 512
    rng = np.random.default_rng(5)
    a = rng.standard_normal(m * n)
    c = np.zeros(n * m)
    LA = gpu.block_cyclic_layout(m, n, b, b, 1, 1, m, n, 1, 1, "R", 0, 0, a, m, "C", 0)
    LC = gpu.block_cyclic_layout(n, m, b, b, 1, 1, n, m, 1, 1, "R", 0, 0, c, n, "C", 0)
    comm = gpu.Comm.self(0)
    exp = a.reshape(n, m).T.copy().reshape(-1)  # C(j, i) = A(i, j): C col i = A row i
    try:
        for k, mode in enumerate([1, 1, 0, 1, 0, 0, 1]):
            gpu.set_host_staging(mode)
            c[:] = np.nan
            a *= -1 if k % 2 else 1
            exp = a.reshape(n, m).T.copy().reshape(-1)
            gpu.transform(LA, LC, comm, "T", 1.0, 0.0)
            assert np.array_equal(c, exp), f"call {k} (mode {mode})"
    finally:
        gpu.set_host_staging(1)


def _pinned_copy(x):
    """a page-locked copy of numpy array x (torch's pinned allocator = hipHostMalloc) and the
    tensor that owns it"""
    t = torch.empty(max(1, x.nbytes), dtype=torch.uint8, pin_memory=True)
    a = t.numpy()[:x.nbytes].view(x.dtype)
    a[:] = x
    return a, t


@pytest.mark.parametrize("case", SINGLE, ids=lambda c: c.name)
def test_golden_host_pinned(gpu, case):
    """host-resident layouts in page-locked memory: the pipeline moves every tile by strided DMA
    between the caller's arrays and HBM (no host gather / scatter) and must match the reference
    bit for bit, C bytes outside the transform untouched"""
    keep, As, Cs = [], [], []
    for k in range(len(case.pairs)):
        a, c = case.inputs(k, 0)
        pa, ta = _pinned_copy(a)
        pc, tc = _pinned_copy(c)
        keep.append((pa, ta, pc, tc))
        As.append(case.layout_A(k, 0, pa.ctypes.data))
        Cs.append(case.layout_C(k, 0, pc.ctypes.data))
    eff = [case.effective(k) for k in range(len(case.pairs))]
    gpu.get_stats(reset=True)
    gpu.transform_batch(As, Cs, gpu.Comm.self(0), [e[0] for e in eff], [e[1] for e in eff],
                        [e[2] for e in eff])
    st = gpu.get_stats(reset=True)
    fx = load(case.name)
    for k in range(len(case.pairs)):
        key = f"C{k}_r0"
        got = keep[k][2]
        assert matches(fx, key, got), f"{case.name} {key}: " + first_mismatch(fx, key, got)
    # direct DMA for the groups whose footprints are rectangles of the caller's arrays, the
    # copying pipeline for the rest, in the same call.  How many groups go direct is fixed by the
    # plan (deterministic): recorded per case in tests/golden/host_direct.json on the GPU
    # (COSTA_RECORD_HOST_DIRECT=<file> writes the counts instead of checking them)
    d = st["host_direct_groups"]
    assert d <= st["host_groups"] and (st["host_direct"] > 0) == (d > 0)
    rec = os.environ.get("COSTA_RECORD_HOST_DIRECT")
    if rec:
        with open(rec, "a") as f:
            f.write(json.dumps({case.name: [int(d), int(st["host_groups"])]}) + "\n")
        return
    assert case.name in DIRECT_EXPECTED, f"{case.name}: no recorded direct-group count"
    assert [d, st["host_groups"]] == DIRECT_EXPECTED[case.name], case.name
    if case.name == "block_cyclic":  # whole block-cyclic matrices: every group is a rectangle
        assert d == st["host_groups"] >= 1


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("trans,alpha,beta", [("T", 1.0, 0.0), ("T", -0.75, 1.5), ("N", 2.0, 0.5)])
def test_large_host_pinned_vs_numpy(gpu, shape, trans, alpha, beta):
    """several 64 MiB groups, pieces of one large block, ragged blocks, with beta != 0 (old C
    values uploaded by DMA too) from page-locked memory; pageable A with pinned C stays on the
    copying pipeline"""
    m, n, mb, nb = shape
    rng = np.random.default_rng(12)
    a0 = rng.standard_normal(m * n)
    cm, cn = (n, m) if trans == "T" else (m, n)
    c0 = rng.standard_normal(cm * cn)
    x = a0.reshape(n, m).T.copy().reshape(-1) if trans == "T" else a0
    exp = alpha * x if beta == 0 else beta * c0 + alpha * x
    cmb, cnb = (nb, mb) if trans == "T" else (mb, nb)
    for pin_a in (True, False):
        a, ta = _pinned_copy(a0) if pin_a else (a0.copy(), None)
        c, tc = _pinned_copy(c0)
        LA = gpu.block_cyclic_layout(m, n, mb, nb, 1, 1, m, n, 1, 1, "R", 0, 0, a, m, "C", 0)
        LC = gpu.block_cyclic_layout(cm, cn, cmb, cnb, 1, 1, cm, cn, 1, 1, "R", 0, 0, c, cm, "C", 0)
        gpu.get_stats(reset=True)
        gpu.transform(LA, LC, gpu.Comm.self(0), trans, alpha, beta)
        st = gpu.get_stats(reset=True)
        assert np.array_equal(c.view(np.uint64), exp.view(np.uint64)), f"pinned A: {pin_a}"
        assert st["host_groups"] >= 1
        assert (st["host_direct"] >= 1) == pin_a
        del LA, LC, ta, tc
