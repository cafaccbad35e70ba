"""GPU: the device planner (costa_amd/csrc/device_plan.hip) against the host
planner (plan.cpp, pinned to the reference by tests/test_plan_cpu.py).

The device planner enumerates the merged grid of each layout pair on the GPU.  Its op lists must
equal the host planner's field for field and in the same order, with the same package counts,
displacements and scalars, for every rank of every golden case and at the BASELINE geometries
(cfg 3, 4, 5 and a sub-matrix case; block addresses there are never dereferenced).  Then whole
transforms with the device planner forced (costa_hip_set_planner(2)) against the golden outputs,
and the host fallback for layouts it does not take."""
import numpy as np
import pytest

from cases import all_cases
from golden_io import first_mismatch, load, matches

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def gpu(costa):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    yield costa
    costa.set_planner(1)


def assert_same(h, d):
    for f in ("local_ops", "pack_ops", "unpack_ops"):
        a, b = getattr(h, f), getattr(d, f)
        assert a.shape == b.shape, f"{f}: {a.shape} vs {b.shape}"
        if a.size and a.tobytes() != b.tobytes():
            bad = np.nonzero(a != b)[0]
            raise AssertionError(f"{f}: {bad.size} ops differ, first #{bad[0]}: host {a[bad[0]]} "
                                 f"device {b[bad[0]]}")
    for f in ("send_counts", "send_displs", "recv_counts", "recv_displs"):
        assert np.array_equal(getattr(h, f), getattr(d, f)), f
    assert (h.send_elems, h.recv_elems, h.local_elems) == (d.send_elems, d.recv_elems,
                                                           d.local_elems)
    assert h.scalars.tobytes() == d.scalars.tobytes()


def both(costa, As, Cs, rank, P, trans, alpha, beta):
    h = costa.plan_export(As, Cs, rank, P, trans, alpha, beta)
    d = costa.plan_export(As, Cs, rank, P, trans, alpha, beta, device=0)
    assert_same(h, d)
    return h


@pytest.mark.parametrize("case", all_cases(), ids=lambda c: c.name)
def test_device_plan_equals_host_golden(gpu, case):
    eff = [case.effective(k) for k in range(len(case.pairs))]
    for r in range(case.P):
        As = [case.layout_A(k, r, (1 << 40) + (k << 34)) for k in range(len(case.pairs))]
        Cs = [case.layout_C(k, r, (1 << 41) + (k << 34)) for k in range(len(case.pairs))]
        both(gpu, As, Cs, r, case.P, [e[0] for e in eff], [e[1] for e in eff],
             [e[2] for e in eff])


def cfg5_layouts(costa, world, rank):
    """BASELINE configs[4] geometry (bench.py cfg5_workload) at fake addresses"""
    n = 16384

    def splits(seed, lo, hi):
        r = np.random.default_rng(seed)
        s = [0]
        while s[-1] < n:
            s.append(min(n, s[-1] + int(r.integers(lo, hi + 1))))
        return s

    def layout(rs, cs, own, base):
        blocks, off = [], 0
        for i in range(len(rs) - 1):
            for j in range(len(cs) - 1):
                if own[i, j] != rank:
                    continue
                rows, cols = rs[i + 1] - rs[i], cs[j + 1] - cs[j]
                blocks.append((base + 4 * off, rows, i, j))
                off += (rows * cols + 63) // 64 * 64
        return costa.custom_layout(len(rs) - 1, len(cs) - 1, rs, cs, own, blocks, "C", costa.FLOAT)

    ars, acs = splits(0xC5A1, 8, 96), splits(0xC5A2, 8, 96)
    crs, ccs = splits(0xC5A3, 16, 160), splits(0xC5A4, 16, 160)
    aown = np.random.default_rng(0xC5A5).integers(0, world, (len(ars) - 1, len(acs) - 1))
    cown = np.random.default_rng(0xC5A6).integers(0, world, (len(crs) - 1, len(ccs) - 1))
    return layout(ars, acs, aown, 1 << 40), layout(crs, ccs, cown, 1 << 41)


@pytest.mark.parametrize("world,rank", [(1, 0), (8, 5)])
@pytest.mark.parametrize("op,ab", [("N", (1.0, 0.0)), ("T", (-0.5, 2.0))])
def test_device_plan_equals_host_cfg5(gpu, world, rank, op, ab):
    LA, LC = cfg5_layouts(gpu, world, rank)
    p = both(gpu, [LA], [LC], rank, world, [op], [ab[0]], [ab[1]])
    n = p.local_ops.size + p.pack_ops.size
    assert n > 200000 // world, n  # the whole tile set of the rank (~242 k tiles over all ranks)


@pytest.mark.parametrize("name", ["cfg3", "cfg4", "submatrix"])
def test_device_plan_equals_host_block_cyclic(gpu, name):
    c = gpu
    if name == "cfg3":  # pxgemr2d fp64 65536^2, 128^2 blocks, 2x2 -> 4x1 'R', rank 1, 'N'
        m = n = 65536
        r, P, args = 1, 4, dict(trans="N", alpha=1.0, beta=0.0)
        A = c.block_cyclic_layout(m, n, 128, 128, 1, 1, m, n, 2, 2, "R", 0, 0, 1 << 40, 32768, "C", r)
        C = c.block_cyclic_layout(m, n, 128, 128, 1, 1, m, n, 4, 1, "R", 0, 0, 1 << 42, 16384, "C", r)
    elif name == "cfg4":  # pztranu c128 32768^2, 128^2 blocks, 2x4 both, rank 3, 'T'
        m = n = 32768
        r, P, args = 3, 8, dict(trans="T", alpha=complex(0.75, -0.5), beta=complex(1.25, 0.25))
        A = c.block_cyclic_layout(m, n, 128, 128, 1, 1, m, n, 2, 4, "R", 0, 0, 1 << 40, 16384, "C",
                                  r, c.CDOUBLE)
        C = c.block_cyclic_layout(m, n, 128, 128, 1, 1, m, n, 2, 4, "R", 0, 0, 1 << 42, 16384, "C",
                                  r, c.CDOUBLE)
    else:  # sub-matrices, row-major storage, rsrc/csrc, mismatched blocks, 'T', rank 4 of 6
        r, P, args = 4, 6, dict(trans="T", alpha=-2.0, beta=0.5)
        A = c.block_cyclic_layout(1000, 900, 64, 48, 5, 7, 700, 650, 2, 3, "C", 1, 2, 1 << 40, 600,
                                  "R", r)
        C = c.block_cyclic_layout(800, 1200, 50, 70, 3, 11, 650, 700, 3, 2, "R", 2, 0, 1 << 41, 400,
                                  "C", r)
    both(c, [A], [C], r, P, [args["trans"]], [args["alpha"]], [args["beta"]])


def _random_splits(rng, n):
    """ragged split points of [0, n), with repeated points (empty block rows / columns)"""
    s = [0]
    while s[-1] < n:
        s.append(min(n, s[-1] + int(rng.integers(1, max(2, n // 3) + 1))))
        if rng.random() < 0.15:
            s.append(s[-1])
    return s


def _random_custom(costa, rng, m, n, P, rank, base, dtype, ordering):
    rs, cs = _random_splits(rng, m), _random_splits(rng, n)
    own = rng.integers(0, P, (len(rs) - 1, len(cs) - 1))
    E = 16
    blocks, off = [], 0
    for i in range(len(rs) - 1):
        for j in range(len(cs) - 1):
            if own[i, j] != rank:
                continue
            rows, cols = rs[i + 1] - rs[i], cs[j + 1] - cs[j]
            ld = (cols if ordering == "R" else rows) + int(rng.integers(0, 3))
            blocks.append((base + E * off, max(ld, 1), i, j))
            off += max(ld, 1) * (rows if ordering == "R" else cols) + 8
    return costa.custom_layout(len(rs) - 1, len(cs) - 1, rs, cs, own, blocks, ordering, dtype)


@pytest.mark.parametrize("seed", range(24))
def test_device_plan_equals_host_random(gpu, seed):
    """random ragged custom layouts (empty block rows / columns, ld padding, both orderings),
    1-5 ranks, every rank, 1-3 layout pairs per batch, every op and scale kind"""
    rng = np.random.default_rng(1000 + seed)
    dtype = int(rng.integers(0, 5))
    P = int(rng.integers(1, 6))
    jobs = []
    for k in range(int(rng.integers(1, 4))):
        m, n = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        op = "NTC"[int(rng.integers(0, 3))]
        cm, cn = (n, m) if op != "N" else (m, n)
        ab = [(1.0, 0.0), (0.0, 0.0), (-0.5, 0.0), (1.0, 1.0), (2.0, -0.25)][int(rng.integers(0, 5))]
        if dtype == gpu.INT32:
            ab = (int(ab[0]), int(ab[1]))
        jobs.append((m, n, cm, cn, op, ab, "RC"[int(rng.integers(0, 2))], "RC"[int(rng.integers(0, 2))],
                     int(rng.integers(0, 1 << 30))))
    for r in range(P):
        As, Cs = [], []
        for k, (m, n, cm, cn, op, ab, oa, oc, s) in enumerate(jobs):
            # the same grids and owners on every rank: the layouts' rng is re-seeded per job
            As.append(_random_custom(gpu, np.random.default_rng(s), m, n, P, r,
                                     (1 << 40) + (k << 34), dtype, oa))
            Cs.append(_random_custom(gpu, np.random.default_rng(s + 1), cm, cn, P, r,
                                     (1 << 41) + (k << 34), dtype, oc))
        both(gpu, As, Cs, r, P, [j[4] for j in jobs], [j[5][0] for j in jobs],
             [j[5][1] for j in jobs])


@pytest.mark.parametrize("case", [c for c in all_cases() if c.P == 1], ids=lambda c: c.name)
def test_transform_with_device_planner(gpu, case):
    """the engine's plan-cache miss through the device planner, end to end"""
    from test_gpu_parity import _run_single_rank
    gpu.set_planner(2)
    gpu.release_caches()  # plans cached by earlier tests were built on the host
    try:
        d0 = gpu.get_stats()["device_plans"]
        got = _run_single_rank(gpu, case)
        assert gpu.get_stats()["device_plans"] > d0
    finally:
        gpu.set_planner(1)
    fx = load(case.name)
    for k in range(len(case.pairs)):
        assert matches(fx, f"C{k}_r0", got[k]), first_mismatch(fx, f"C{k}_r0", got[k])


def test_device_planner_declines_foreign_blocks(gpu):
    """local blocks that the owner matrix gives to another rank (the host planner takes them:
    it decomposes whatever blocks a layout lists) go to the host planner"""
    rs = [0, 4, 8]
    own = [[1, 1], [1, 1]]

    def blocks(base):
        return [(base + 128 * (2 * i + j), 4, i, j) for i in range(2) for j in range(2)]

    A = gpu.custom_layout(2, 2, rs, rs, own, blocks(1 << 40), "C")
    C = gpu.custom_layout(2, 2, rs, rs, own, blocks(1 << 41), "C")
    with pytest.raises(gpu.CostaError, match="device planner"):
        gpu.plan_export([A], [C], 0, 2, device=0)
    h = gpu.plan_export([A], [C], 0, 2)
    assert h.pack_ops.size == 4 and h.unpack_ops.size == 4 and h.local_ops.size == 0
