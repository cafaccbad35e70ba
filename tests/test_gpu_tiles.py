"""GPU parity of one batched tile launch against the oracle, on random op lists that mix every
work class of the executor: tiny ops (one wavefront each, copy and LDS transpose), the medium
and large sub-tile shapes (copy and transposing lists), the class boundaries (engine.cpp tiny_copy_budget / kTinyLdsBytes), thin
ops (nf = 1, ns = 1), padded strides, unaligned offsets, and every scale kind.

Each op is the reference's copy_and_transform (memory_utils.hpp:339-412); the oracle executes
the same list op by op (oracle.exec_tile_ops).  Bit-exact: integers and finite floats with
contraction off on both sides.
"""
import numpy as np
import pytest

import costa_amd
import oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

TINY_LDS = 4096  # engine.hpp kTinyLdsDefault


def tiny_copy(E, local=True):
    """engine.cpp tiny_copy_budget: half a wavefront pass for local lists (32 lanes x
    tiny_copy_lane_bytes), 3/4 for pack / unpack lists (48 lanes)"""
    return (32 if local else 48) * 64


@pytest.fixture(scope="module")
def gpu(costa):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return costa


def _values(rng, dt, n):
    if dt == np.int32:
        return rng.integers(-1000, 1000, n, dtype=np.int32)
    x = rng.standard_normal(n)
    if np.issubdtype(dt, np.complexfloating):
        x = x + 1j * rng.standard_normal(n)
    return x.astype(dt)


def _shape(rng, E, transpose):
    """(nf, ns) drawn to hit every class and the boundaries between them"""
    pick = rng.integers(0, 8)
    if pick == 0:  # tiny, ragged
        return int(rng.integers(1, 70)), int(rng.integers(1, 70))
    if pick == 1:  # at the tiny boundary
        limit = (TINY_LDS if transpose else tiny_copy(E, bool(rng.integers(0, 2)))) // E
        nf = int(rng.integers(1, 129))
        ns = max(1, limit // ((nf | 1) if transpose else nf) + int(rng.integers(-1, 2)))
        return nf, ns
    if pick == 2:  # thin column
        return 1, int(rng.integers(1, 5000))
    if pick == 3:  # thin row
        return int(rng.integers(1, 5000)), 1
    if pick == 4:  # medium (small shape)
        return int(rng.integers(60, 200)), int(rng.integers(40, 140))
    if pick == 5:  # large shape, ragged edge
        return int(rng.integers(200, 600)), int(rng.integers(100, 300))
    if pick == 6:  # around the medium shape (256 threads, 16 KiB sub-tiles) of transposing lists
        return int(rng.integers(16, 100)), int(rng.integers(16, 100))
    return int(rng.integers(1, 400)), int(rng.integers(1, 400))


def _random_list(rng, code, n_ops, copy_only=False):
    """op list whose scale kinds agree with the slot scalars (see SLOTS); copy_only: no
    transposing op (the executor then runs large ops on its copy shape)"""
    dt = oracle.NP[code]
    E = np.dtype(dt).itemsize
    cplx = np.issubdtype(dt, np.complexfloating)
    ops = np.zeros(n_ops, costa_amd.TILE_OP_DTYPE)
    src_off = dst_off = 0
    for i in range(n_ops):
        tr = bool(rng.integers(0, 2)) and not copy_only
        nf, ns = _shape(rng, E, tr)
        lds = nf + int(rng.integers(0, 2)) * int(rng.integers(0, 5))
        dn = ns if tr else nf
        ldd = dn + int(rng.integers(0, 2)) * int(rng.integers(0, 5))
        d_slow = nf if tr else ns
        if rng.integers(0, 3) == 0:  # misalign the start by a few elements
            src_off += int(rng.integers(1, 4))
            dst_off += int(rng.integers(1, 4))
        else:  # 16-byte aligned
            src_off = -(-src_off * E // 16) * 16 // E
            dst_off = -(-dst_off * E // 16) * 16 // E
        conj = bool(cplx and rng.integers(0, 2))
        kind = int(rng.integers(0, 4))
        if kind == 0 and (tr or conj):  # the planner never bit-copies through a transpose/conj
            kind = 2
            slot = 0  # alpha = 1, beta = 0 evaluated as a product (memory_utils.hpp:101-291)
        else:
            slot = (0, 1, 2, 3)[kind] if kind != 2 else int(rng.choice([0, 2]))
        flags = (1 if tr else 0) | (2 if conj else 0) | (kind << 4) | (slot << 16)
        if (src_off * E) % 16 == 0 and (lds * E) % 16 == 0:
            flags |= 4
        if (dst_off * E) % 16 == 0 and (ldd * E) % 16 == 0:
            flags |= 8
        ops[i] = (src_off * E, dst_off * E, nf, ns, lds, ldd, flags, 0)
        src_off += (ns - 1) * lds + nf
        dst_off += (d_slow - 1) * ldd + dn
    return ops, src_off, dst_off


@pytest.mark.parametrize("code", [0, 1, 2, 3, 4], ids=["f32", "f64", "c64", "c128", "i32"])
@pytest.mark.parametrize("seed", [1, 2, 3, "copy"])
def test_mixed_tile_list(gpu, code, seed):
    copy_only = seed == "copy"
    rng = np.random.default_rng(1000 * (7 if copy_only else seed) + code)
    dt = oracle.NP[code]
    ops, n_src, n_dst = _random_list(rng, code, 240, copy_only)
    src = _values(rng, dt, n_src)
    dst0 = _values(rng, dt, n_dst)
    # SLOTS: 0 = (1, 0) bit copy / unit scale, 1 = (0, 0), 2 = (alpha, 0), 3 = (alpha, beta)
    if dt == np.int32:
        scal = np.array([1, 0, 0, 0, 2, 0, -3, 5], dt)
    else:
        a, b = _values(rng, dt, 2)
        scal = np.array([1, 0, 0, 0, a, 0, a, b], dt)
    exp = dst0.copy()
    oracle.exec_tile_ops(code, ops, scal, src.ctypes.data, exp.ctypes.data)

    d_src = torch.from_numpy(src.view(np.uint8).copy()).cuda()
    d_dst = torch.from_numpy(dst0.view(np.uint8).copy()).cuda()
    gpu.execute_tiles(code, ops, scal, d_src.data_ptr(), d_dst.data_ptr())
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy().view(dt)
    E = np.dtype(dt).itemsize
    bad = np.flatnonzero((got.view(np.uint8).reshape(n_dst, E)
                          != exp.view(np.uint8).reshape(n_dst, E)).any(1))
    assert bad.size == 0, f"{bad.size} elements differ, first at {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"


@pytest.mark.parametrize("code,nb,full", [(0, 64, False), (1, 32, False), (1, 48, False), (4, 64, False),
                                          (0, 80, False), (0, 64, True), (4, 64, True), (0, 32, False),
                                          (2, 32, False), (3, 32, False), (4, 24, False)],
                         ids=["f32-64", "f64-32", "f64-48", "i32-64", "f32-80", "f32-64-full", "i32-64-full",
                              "f32-32", "c64-32", "c128-32", "i32-24"])
def test_medium_shape_list(gpu, code, nb, full):
    """a transposing list of >= 4096 aligned ops between half a medium and half a large
    sub-tile (engine.cpp kMinMediumOps: the medium shape only runs for lists this long), with
    every scale kind and padded strides; full: every op a whole medium sub-tile (the
    `medium_tr_full` launch); nb <= 32: the medium class on 32 x 32 sub-tiles (`small32_tr`,
    every type); bit-exact against the oracle"""
    rng = np.random.default_rng(77 + code + nb)
    dt = oracle.NP[code]
    E = np.dtype(dt).itemsize
    n_ops = 4200
    ops = np.zeros(n_ops, costa_amd.TILE_OP_DTYPE)
    src_off = dst_off = 0
    for i in range(n_ops):
        # full, or (above 32) one 16-byte vector short: every op stays in the medium class
        nf = nb - (int(rng.integers(0, 2)) * (16 // E) if nb > 32 and not full else 0)
        ns = nb
        if nb == 32 and rng.integers(0, 25) == 0:  # a few partly filled 32 x 32 sub-tiles
            nf, ns = int(rng.integers(17, 33)), int(rng.integers(17, 33))
        lds = nf + int(rng.integers(0, 2)) * (16 // E)
        ldd = ns + int(rng.integers(0, 2)) * (16 // E)
        kind = int(rng.integers(1, 3 if full else 4))  # full: no C read (the 128-thread launch)
        slot = (0, 1, 2, 3)[kind] if kind != 2 else int(rng.choice([0, 2]))
        ops[i] = (src_off * E, dst_off * E, nf, ns, lds, ldd, 1 | 4 | 8 | (kind << 4) | (slot << 16), 0)
        src_off += -(-((ns - 1) * lds + nf) * E // 16) * 16 // E
        dst_off += -(-((nf - 1) * ldd + ns) * E // 16) * 16 // E
    src = _values(rng, dt, src_off)
    dst0 = _values(rng, dt, dst_off)
    if dt == np.int32:
        scal = np.array([1, 0, 0, 0, 2, 0, -3, 5], dt)
    else:
        a, b = _values(rng, dt, 2)
        scal = np.array([1, 0, 0, 0, a, 0, a, b], dt)
    exp = dst0.copy()
    oracle.exec_tile_ops(code, ops, scal, src.ctypes.data, exp.ctypes.data)
    d_src = torch.from_numpy(src.view(np.uint8).copy()).cuda()
    d_dst = torch.from_numpy(dst0.view(np.uint8).copy()).cuda()
    gpu.execute_tiles(code, ops, scal, d_src.data_ptr(), d_dst.data_ptr())
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy().view(dt)
    bad = np.flatnonzero((got.view(np.uint8).reshape(dst_off, E)
                          != exp.view(np.uint8).reshape(dst_off, E)).any(1))
    assert bad.size == 0, f"{bad.size} elements differ, first at {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"


@pytest.mark.parametrize("code", [0, 1, 2, 3, 4], ids=["f32", "f64", "c64", "c128", "i32"])
@pytest.mark.parametrize("copy_only", [False, True], ids=["mixed", "copy"])
def test_unaligned_large_list(gpu, code, copy_only):
    """large ops whose columns are not 16-byte aligned on one side or both (odd lld for 8-byte
    types, lld % 4 != 0 for 4-byte ones): the large shape's element-wise path
    (tile_kernels.hip run_tile_elem), full and ragged sub-tiles, every scale kind; bit-exact
    against the oracle"""
    rng = np.random.default_rng(4242 + code + 10 * copy_only)
    dt = oracle.NP[code]
    E = np.dtype(dt).itemsize
    cplx = np.issubdtype(dt, np.complexfloating)
    n_ops = 40
    ops = np.zeros(n_ops, costa_amd.TILE_OP_DTYPE)
    src_off = dst_off = 0
    for i in range(n_ops):
        tr = bool(rng.integers(0, 2)) and not copy_only
        nf, ns = int(rng.integers(100, 420)), int(rng.integers(100, 300))
        side = int(rng.integers(0, 3))  # 0: source unaligned, 1: destination, 2: both
        lds = nf + (int(rng.integers(0, 3)) * 2 + 1 if side != 1 else 16 // E)
        dn, d_slow = (ns, nf) if tr else (nf, ns)
        ldd = dn + (int(rng.integers(0, 3)) * 2 + 1 if side != 0 else 16 // E)
        src_off = -(-src_off * E // 16) * 16 // E + (int(rng.integers(0, 2)) if side != 1 else 0)
        dst_off = -(-dst_off * E // 16) * 16 // E + (int(rng.integers(0, 2)) if side != 0 else 0)
        conj = bool(cplx and rng.integers(0, 2))
        kind = int(rng.integers(0, 4))
        if kind == 0 and (tr or conj):
            kind = 2
            slot = 0
        else:
            slot = (0, 1, 2, 3)[kind] if kind != 2 else int(rng.choice([0, 2]))
        flags = (1 if tr else 0) | (2 if conj else 0) | (kind << 4) | (slot << 16)
        if (src_off * E) % 16 == 0 and (lds * E) % 16 == 0:
            flags |= 4
        if (dst_off * E) % 16 == 0 and (ldd * E) % 16 == 0:
            flags |= 8
        ops[i] = (src_off * E, dst_off * E, nf, ns, lds, ldd, flags, 0)
        src_off += (ns - 1) * lds + nf
        dst_off += (d_slow - 1) * ldd + dn
    src = _values(rng, dt, src_off)
    dst0 = _values(rng, dt, dst_off)
    if dt == np.int32:
        scal = np.array([1, 0, 0, 0, 2, 0, -3, 5], dt)
    else:
        a, b = _values(rng, dt, 2)
        scal = np.array([1, 0, 0, 0, a, 0, a, b], dt)
    exp = dst0.copy()
    oracle.exec_tile_ops(code, ops, scal, src.ctypes.data, exp.ctypes.data)
    d_src = torch.from_numpy(src.view(np.uint8).copy()).cuda()
    d_dst = torch.from_numpy(dst0.view(np.uint8).copy()).cuda()
    gpu.execute_tiles(code, ops, scal, d_src.data_ptr(), d_dst.data_ptr())
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy().view(dt)
    bad = np.flatnonzero((got.view(np.uint8).reshape(dst_off, E)
                          != exp.view(np.uint8).reshape(dst_off, E)).any(1))
    assert bad.size == 0, f"{bad.size} elements differ, first at {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"


@pytest.mark.parametrize("code", [1, 2, 3], ids=["f64", "c64", "c128"])
@pytest.mark.parametrize("seed", [1, 2])
def test_square_shape_list(gpu, code, seed):
    """a transposing list whose large ops all fit 64 x 64 (nb = 64 blocks): the large ops run on
    the square variant of the transposing shape (engine.cpp build_work, tile_kernels.hip
    small_tr); copy-mode ops, padded and unaligned strides, every scale kind (conjugation for
    complex types), plus small ops on the wavefront path; bit-exact against the oracle"""
    rng = np.random.default_rng(640 + seed + 10 * code)
    dt = oracle.NP[code]
    E = np.dtype(dt).itemsize
    cplx = np.issubdtype(dt, np.complexfloating)
    n_ops = 600
    ops = np.zeros(n_ops, costa_amd.TILE_OP_DTYPE)
    src_off = dst_off = 0
    for i in range(n_ops):
        tr = rng.integers(0, 4) != 0
        nf, ns = ((64, 64) if rng.integers(0, 3) else (int(rng.integers(46, 65)), int(rng.integers(46, 65)))) \
            if rng.integers(0, 5) else (int(rng.integers(1, 40)), int(rng.integers(1, 40)))
        lds = nf + int(rng.integers(0, 3)) * int(rng.integers(0, 2))
        dn, d_slow = (ns, nf) if tr else (nf, ns)
        ldd = dn + int(rng.integers(0, 3)) * int(rng.integers(0, 2))
        if rng.integers(0, 4) == 0:
            src_off += 1
            dst_off += 1
        else:
            src_off = -(-src_off * E // 16) * 16 // E
            dst_off = -(-dst_off * E // 16) * 16 // E
        conj = bool(cplx and rng.integers(0, 2))
        kind = int(rng.integers(0, 4))
        if kind == 0 and (tr or conj):
            kind, slot = 2, 0
        else:
            slot = (0, 1, 2, 3)[kind] if kind != 2 else int(rng.choice([0, 2]))
        flags = (1 if tr else 0) | (2 if conj else 0) | (kind << 4) | (slot << 16)
        if (src_off * E) % 16 == 0 and (lds * E) % 16 == 0:
            flags |= 4
        if (dst_off * E) % 16 == 0 and (ldd * E) % 16 == 0:
            flags |= 8
        ops[i] = (src_off * E, dst_off * E, nf, ns, lds, ldd, flags, 0)
        src_off += (ns - 1) * lds + nf
        dst_off += (d_slow - 1) * ldd + dn
    src = _values(rng, dt, src_off)
    dst0 = _values(rng, dt, dst_off)
    a, b = _values(rng, dt, 2)
    scal = np.array([1, 0, 0, 0, a, 0, a, b], dt)
    exp = dst0.copy()
    oracle.exec_tile_ops(code, ops, scal, src.ctypes.data, exp.ctypes.data)
    d_src = torch.from_numpy(src.view(np.uint8).copy()).cuda()
    d_dst = torch.from_numpy(dst0.view(np.uint8).copy()).cuda()
    gpu.execute_tiles(code, ops, scal, d_src.data_ptr(), d_dst.data_ptr())
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy().view(dt)
    bad = np.flatnonzero((got.view(np.uint8).reshape(dst_off, E)
                          != exp.view(np.uint8).reshape(dst_off, E)).any(1))
    assert bad.size == 0, f"{bad.size} elements differ, first at {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"


@pytest.mark.parametrize("code", [3, 1], ids=["c128", "f64"])
def test_full_tile_list(gpu, code):
    """a transposing list whose ops are all aligned whole multiples of the large sub-tile (c128
    64 x 128, fp64 64 x 128): the `large_tr_full` launch (engine.cpp work_split::full); copy and
    transpose ops, every scale kind (conjugation for c128); bit-exact against the oracle"""
    rng = np.random.default_rng(9100 + code)
    dt = oracle.NP[code]
    E = np.dtype(dt).itemsize
    cplx = np.issubdtype(dt, np.complexfloating)
    n_ops = 40
    ops = np.zeros(n_ops, costa_amd.TILE_OP_DTYPE)
    src_off = dst_off = 0
    for i in range(n_ops):
        tr = i == 0 or rng.integers(0, 4) != 0
        nf, ns = 64 * int(rng.integers(1, 4)), 128 * int(rng.integers(1, 3))
        lds = nf + (16 // E) * int(rng.integers(0, 2))
        dn, d_slow = (ns, nf) if tr else (nf, ns)
        ldd = dn + (16 // E) * int(rng.integers(0, 2))
        conj = bool(cplx and rng.integers(0, 2))
        kind = int(rng.integers(0, 4))
        if kind == 0 and (tr or conj):
            kind, slot = 2, 0
        else:
            slot = (0, 1, 2, 3)[kind] if kind != 2 else int(rng.choice([0, 2]))
        ops[i] = (src_off * E, dst_off * E, nf, ns, lds, ldd,
                  (1 if tr else 0) | (2 if conj else 0) | 4 | 8 | (kind << 4) | (slot << 16), 0)
        src_off += -(-((ns - 1) * lds + nf) * E // 16) * 16 // E
        dst_off += -(-((d_slow - 1) * ldd + dn) * E // 16) * 16 // E
    src = _values(rng, dt, src_off)
    dst0 = _values(rng, dt, dst_off)
    a, b = _values(rng, dt, 2)
    scal = np.array([1, 0, 0, 0, a, 0, a, b], dt)
    exp = dst0.copy()
    oracle.exec_tile_ops(code, ops, scal, src.ctypes.data, exp.ctypes.data)
    d_src = torch.from_numpy(src.view(np.uint8).copy()).cuda()
    d_dst = torch.from_numpy(dst0.view(np.uint8).copy()).cuda()
    gpu.execute_tiles(code, ops, scal, d_src.data_ptr(), d_dst.data_ptr())
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy().view(dt)
    bad = np.flatnonzero((got.view(np.uint8).reshape(dst_off, E)
                          != exp.view(np.uint8).reshape(dst_off, E)).any(1))
    assert bad.size == 0, f"{bad.size} elements differ, first at {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"


@pytest.mark.parametrize("code", [0, 4], ids=["f32", "i32"])
@pytest.mark.parametrize("seed", [1, 2])
def test_wavefront_transposes_every_phase(gpu, code, seed):
    """wavefront transposes of 4-byte elements into destination columns at every 16-byte phase
    (r4 measured a variant that writes aligned 16-byte chunks with element-wise heads and tails;
    this pins the edges any such variant must get right): every destination offset mod 4, leading dimensions ns .. ns + 3 (each column starting at
    another phase), heights 1 .. 160 (all edges, no full chunk, a single chunk), widths 1 .. 64,
    ops the host cuts into pieces, every scale kind; neighbouring ops' destination columns share
    16-byte chunks (no op may write outside its own elements).  Bit-exact against the oracle."""
    rng = np.random.default_rng(9300 + 10 * seed + code)
    dt = oracle.NP[code]
    E = np.dtype(dt).itemsize
    n_ops = 600
    ops = np.zeros(n_ops, costa_amd.TILE_OP_DTYPE)
    src_off = dst_off = 0
    for i in range(n_ops):
        nf = int(rng.integers(1, 65))
        ns = int(rng.choice([int(rng.integers(1, 12)), int(rng.integers(8, 161))]))
        lds = nf + int(rng.integers(0, 4))
        ldd = ns + int(rng.integers(0, 4))
        src_off += int(rng.integers(0, 4))
        dst_off += int(rng.integers(0, 4))
        kind = int(rng.integers(1, 4))
        slot = (0, 1, 2, 3)[kind] if kind != 2 else int(rng.choice([0, 2]))
        flags = 1 | (kind << 4) | (slot << 16)
        if (src_off * E) % 16 == 0 and (lds * E) % 16 == 0:
            flags |= 4
        if (dst_off * E) % 16 == 0 and (ldd * E) % 16 == 0:
            flags |= 8
        ops[i] = (src_off * E, dst_off * E, nf, ns, lds, ldd, flags, 0)
        src_off += (ns - 1) * lds + nf
        # the next op's destination starts inside this op's last column's padding (ldd > ns) or
        # right after it: 16-byte chunks are shared between ops
        dst_off += (nf - 1) * ldd + ns
    src = _values(rng, dt, src_off)
    dst0 = _values(rng, dt, dst_off + 8)
    if dt == np.int32:
        scal = np.array([1, 0, 0, 0, 2, 0, -3, 5], dt)
    else:
        a, b = _values(rng, dt, 2)
        scal = np.array([1, 0, 0, 0, a, 0, a, b], dt)
    exp = dst0.copy()
    oracle.exec_tile_ops(code, ops, scal, src.ctypes.data, exp.ctypes.data)
    d_src = torch.from_numpy(src.view(np.uint8).copy()).cuda()
    d_dst = torch.from_numpy(dst0.view(np.uint8).copy()).cuda()
    gpu.execute_tiles(code, ops, scal, d_src.data_ptr(), d_dst.data_ptr())
    torch.cuda.synchronize()
    got = d_dst.cpu().numpy().view(dt)
    n = dst0.size
    bad = np.flatnonzero((got.view(np.uint8).reshape(n, E) != exp.view(np.uint8).reshape(n, E)).any(1))
    assert bad.size == 0, f"{bad.size} elements differ, first at {bad[0]}: {got[bad[0]]} vs {exp[bad[0]]}"
