"""GPU: the work lists' destination-block groups built on the GPU (costa_amd/csrc/device_lists.hip,
SURVEY §8(f)1) against the host builder (engine.cpp cblock_groups, pinned on the CPU by
test_work_lists.py / tools/work_check.cpp).

The two builders must give the same work lists byte for byte -- the ordered op list ([shaped ops |
group headers and ops cut at band edges | wavefront pieces]), the work items and every count of the
split -- for BASELINE cfg 5's lists (242 k tiles, 'N' and 'T', one and eight ranks), every golden
case's local / pack / unpack lists, random ragged layouts, and hand-made lists that probe the
exactness test: components whose areas add up while their ops overlap, mixed transforms, one op
missing, ranges cut into many column bands, lists without locality hints.  Then whole transforms
with the GPU builder forced (costa_hip_set_list_builder(2)) against the golden outputs and the
oracle, with the statistics showing that the GPU built the groups."""
import numpy as np
import pytest

import costa_amd
from cases import all_cases
from golden_io import first_mismatch, load, matches
from test_gpu_device_plan import _random_custom, cfg5_layouts

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

TR, VEC_SRC, VEC_DST = costa_amd.TILE_TRANSPOSE, costa_amd.TILE_VEC_SRC, costa_amd.TILE_VEC_DST
E_OF = {costa_amd.FLOAT: 4, costa_amd.DOUBLE: 8, costa_amd.CFLOAT: 8, costa_amd.CDOUBLE: 16,
        costa_amd.INT32: 4}


@pytest.fixture(scope="module")
def gpu(costa):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    yield costa
    costa.set_list_builder(1)


def same_lists(costa, dtype, ops, kind="local", want_gpu=None):
    """host and GPU work lists of one op list, asserted equal; -> the GPU's"""
    h = costa.work_export(dtype, ops, kind)
    d = costa.work_export(dtype, ops, kind, device=0)
    assert not h.on_gpu
    mh = {k: v for k, v in h.meta.items() if k != "on_gpu"}
    md = {k: v for k, v in d.meta.items() if k != "on_gpu"}
    assert mh == md, f"split differs: host {mh} gpu {md}"
    if h.ordered.tobytes() != d.ordered.tobytes():
        bad = np.nonzero(h.ordered != d.ordered)[0]
        raise AssertionError(f"{bad.size} ordered entries differ, first #{bad[0]}: host "
                             f"{h.ordered[bad[0]]} gpu {d.ordered[bad[0]]}")
    assert h.work.tobytes() == d.work.tobytes(), "work items differ"
    if want_gpu is not None:
        assert d.on_gpu == want_gpu, d.meta
    return d


@pytest.mark.parametrize("world,rank", [(1, 0), (8, 5)])
@pytest.mark.parametrize("op,ab", [("N", (1.0, 0.0)), ("T", (-0.5, 2.0))])
def test_cfg5_lists(gpu, world, rank, op, ab):
    LA, LC = cfg5_layouts(gpu, world, rank)
    p = gpu.plan_export([LA], [LC], rank, world, [op], [ab[0]], [ab[1]])
    d = same_lists(gpu, gpu.FLOAT, p.local_ops, "local", want_gpu=True)
    assert d.meta["n_cblock"] > (50000 if world == 1 else 20), d.meta
    assert d.meta["cb_map"] == (2 if op == "N" else 1)
    if world > 1:
        same_lists(gpu, gpu.FLOAT, p.unpack_ops, "unpack")
        same_lists(gpu, gpu.FLOAT, p.pack_ops, "pack", want_gpu=False)  # packs never group


@pytest.mark.parametrize("case", all_cases(), ids=lambda c: c.name)
def test_golden_lists(gpu, case):
    eff = [case.effective(k) for k in range(len(case.pairs))]
    for r in range(case.P):
        As = [case.layout_A(k, r, (1 << 40) + (k << 34)) for k in range(len(case.pairs))]
        Cs = [case.layout_C(k, r, (1 << 41) + (k << 34)) for k in range(len(case.pairs))]
        p = gpu.plan_export(As, Cs, r, case.P, [e[0] for e in eff], [e[1] for e in eff],
                            [e[2] for e in eff])
        dt = As[0].dtype
        for kind, ops in (("local", p.local_ops), ("pack", p.pack_ops), ("unpack", p.unpack_ops)):
            same_lists(gpu, dt, ops, kind)


@pytest.mark.parametrize("seed", range(16))
def test_random_lists(gpu, seed):
    rng = np.random.default_rng(2000 + seed)
    dtype = int(rng.integers(0, 5))
    P = int(rng.integers(1, 4))
    m, n = int(rng.integers(50, 700)), int(rng.integers(50, 700))
    op = "NTC"[int(rng.integers(0, 3))]
    cm, cn = (n, m) if op != "N" else (m, n)
    ab = [(1.0, 0.0), (-0.5, 0.0), (2.0, -0.25)][int(rng.integers(0, 3))]
    if dtype == gpu.INT32:
        ab = (int(ab[0]), int(ab[1]))
    s = int(rng.integers(0, 1 << 30))
    for r in range(P):
        A = _random_custom(gpu, np.random.default_rng(s), m, n, P, r, 1 << 40, dtype, "C")
        C = _random_custom(gpu, np.random.default_rng(s + 1), cm, cn, P, r, 1 << 41, dtype,
                           "RC"[int(rng.integers(0, 2))])
        p = gpu.plan_export([A], [C], r, P, [op], [ab[0]], [ab[1]])
        for kind, ops in (("local", p.local_ops), ("unpack", p.unpack_ops)):
            same_lists(gpu, dtype, ops, kind)


def _guillotine(rng, r0, r1, c0, c1, max_area, out):
    """random guillotine cuts of [r0, r1) x [c0, c1) into rectangles of at most max_area"""
    h, w = r1 - r0, c1 - c0
    if h * w <= max_area or (h == 1 and w == 1):
        out.append((r0, r1, c0, c1))
        return
    if (w >= h or h == 1) and w > 1:
        c = int(rng.integers(c0 + 1, c1))
        _guillotine(rng, r0, r1, c0, c, max_area, out)
        _guillotine(rng, r0, r1, c, c1, max_area, out)
    else:
        r = int(rng.integers(r0 + 1, r1))
        _guillotine(rng, r0, r, c0, c1, max_area, out)
        _guillotine(rng, r, r1, c0, c1, max_area, out)


def _op(E, base, R, rect, tr, src, lds, hint, kind=2):
    """the tile op writing rectangle (r0, r1, c0, c1) of an R-row column-major range at `base`"""
    r0, r1, c0, c1 = rect
    dst = base + (c0 * R + r0) * E
    run, runs = r1 - r0, c1 - c0
    nf, ns = (runs, run) if tr else (run, runs)
    f = (TR if tr else 0) | (kind << 4)
    if src % 16 == 0 and (lds * E) % 16 == 0:
        f |= VEC_SRC
    if dst % 16 == 0 and (R * E) % 16 == 0:
        f |= VEC_DST
    return (src, dst, nf, ns, lds, R, f, hint)


def _synthetic(seed, E, tr, n_ranges=400, hints=True, corrupt=True):
    """ops tiling n_ranges destination ranges (R rows x K columns, R and K random, several ranges
    back to back in one buffer), some ranges corrupted so that they must not group"""
    rng = np.random.default_rng(seed)
    ops, base = [], 1 << 40
    src = 1 << 36
    for g in range(n_ranges):
        R = int(rng.choice([3, 7, 16, 24, 60, 100, 257, 1000]))
        K = int(rng.integers(1, 400 if R < 100 else 40))
        rects = []
        _guillotine(rng, 0, R, 0, K, int(rng.choice([16, 64, 300, 2000])), rects)
        gap = int(rng.choice([0, 0, 0, 1, 5]))  # a gap in the buffer ends the component
        mode = int(rng.integers(0, 8)) if corrupt else 0
        cur = []
        for i, rect in enumerate(rects):
            lds = int(rng.choice([64, 100, 4096]))
            cur.append(list(_op(E, base, R, rect, tr, src, lds,
                                int(rng.integers(1, 1 << 20)) if hints else 0)))
            src += 1 << 20
        if mode == 1 and len(cur) > 1:      # one op a row down: overlap + gap, same area
            o = cur[int(rng.integers(0, len(cur)))]
            run = o[3] if tr else o[2]
            if run < R:
                o[1] += E
        elif mode == 2 and len(cur) > 1:    # one op with another transform
            cur[int(rng.integers(0, len(cur)))][6] ^= 1 << 4
        elif mode == 3 and len(cur) > 2:    # one op missing
            cur.pop(int(rng.integers(0, len(cur))))
        elif mode == 4 and len(cur) > 1:    # an op twice (areas no longer add up)
            cur.append(list(cur[0]))
        ops += [tuple(o) for o in cur]
        base += (R * K + gap) * E
    a = np.array(ops, dtype=costa_amd.TILE_OP_DTYPE)
    return a[np.random.default_rng(seed + 1).permutation(a.size)]  # list order != destination order


@pytest.mark.parametrize("dtype", [costa_amd.FLOAT, costa_amd.DOUBLE, costa_amd.INT32])
@pytest.mark.parametrize("tr", [False, True])
@pytest.mark.parametrize("hints", [True, False])
@pytest.mark.parametrize("seed", [1, 2])
def test_synthetic_lists(gpu, dtype, tr, hints, seed):
    ops = _synthetic(seed * 10 + dtype, E_OF[dtype], tr, hints=hints)
    d = same_lists(gpu, dtype, ops)
    assert d.meta["n_cblock"] > 50, d.meta
    if not tr and hints:
        assert d.meta["cb_map"] == 2  # the XCD slices of a copy-only list with hints


def test_lists_without_groups(gpu):
    """lists whose ranges all fail the exactness test, and lists of fewer than two candidates"""
    ops = _synthetic(7, 4, False, n_ranges=50, corrupt=False)
    ops["ldd"] = 5000  # past the group budget: no candidate
    d = same_lists(gpu, costa_amd.FLOAT, ops)
    assert d.meta["n_cblock"] == 0 and not d.on_gpu
    same_lists(gpu, costa_amd.FLOAT, ops[:1])
    same_lists(gpu, costa_amd.FLOAT, ops[:0])


@pytest.mark.parametrize("case", [c for c in all_cases() if c.P == 1], ids=lambda c: c.name)
def test_transform_with_gpu_lists(gpu, case):
    """the engine's plan-cache miss with the groups built on the GPU, end to end"""
    from test_gpu_parity import _run_single_rank
    gpu.set_list_builder(2)
    gpu.release_caches()
    try:
        got = _run_single_rank(gpu, case)
    finally:
        gpu.set_list_builder(1)
    fx = load(case.name)
    for k in range(len(case.pairs)):
        assert matches(fx, f"C{k}_r0", got[k]), first_mismatch(fx, f"C{k}_r0", got[k])


@pytest.mark.parametrize("gap", [0, 3])
@pytest.mark.parametrize("op,alpha,beta", [("T", -0.5, 2.0), ("N", 1.0, 0.0)])
def test_cblock_with_gpu_lists(gpu, op, alpha, beta, gap):
    """test_gpu_cblock's ragged custom layouts with the groups built on the GPU: bit-exact against
    the oracle, and the statistics count the GPU-built list"""
    import oracle
    from test_gpu_cblock import test_cblock_vs_oracle
    gpu.set_list_builder(2)
    gpu.release_caches()
    try:
        d0 = gpu.get_stats()["device_lists"]
        test_cblock_vs_oracle(gpu, oracle.FLOAT, op, alpha, beta, gap)
        assert gpu.get_stats()["device_lists"] > d0
    finally:
        gpu.set_list_builder(1)
