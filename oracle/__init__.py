"""TEST INFRASTRUCTURE ONLY — Python access to the CPU oracle (oracle/costa_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this package,
and only as the checker / the timed CPU baseline.  costa_amd never imports it.

Also holds the synthetic-data generator shared with oracle/ref_harness.cpp (splitmix64,
SURVEY §8d), so fixtures made by the reference can be regenerated bit-exactly.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
_lib = None

FLOAT, DOUBLE, CFLOAT, CDOUBLE, INT32 = 0, 1, 2, 3, 4
NP = {FLOAT: np.float32, DOUBLE: np.float64, CFLOAT: np.complex64, CDOUBLE: np.complex128,
      INT32: np.int32}


def build():
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, i, ll = C.c_void_p, C.c_int, C.c_longlong
        L.oracle_copy_and_transform.argtypes = [i, i, i, vp, i, i, vp, i, i, i, i, vp, vp]
        L.oracle_copy_and_transform.restype = None
        L.oracle_bc_table.argtypes = [i, i, i, i, i, i, i, i, i, i, C.c_char, i, i, i, C.c_char,
                                      vp, vp, vp]
        L.oracle_bc_table.restype = ll
        L.oracle_numroc.argtypes = [i, i, i, i, i]
        L.oracle_numroc.restype = i
        L.oracle_transform.argtypes = [i, C.c_char, vp, vp, i, i, vp, vp, vp, i, vp,
                                       i, i, vp, vp, vp, i, vp]
        L.oracle_transform.restype = i
        L.oracle_transform_tiles.argtypes = [i, i, i, vp, vp, vp, vp, vp, ll, i]
        L.oracle_transform_tiles.restype = i
        L.oracle_cmul.argtypes = [i, vp, vp, vp]
        L.oracle_cmul.restype = None
        _lib = L
    return _lib


def scalar(code, x) -> bytes:
    return np.asarray(x, dtype=NP[code]).reshape(1).tobytes()


# ------------------------------------------------------------------ data generator
_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x += np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def _draw(seed: int, rank: int, k: np.ndarray) -> np.ndarray:
    base = np.uint64(seed) ^ (np.uint64(rank) << np.uint64(48))
    return splitmix64(k.astype(np.uint64) ^ base)


def _unif(z: np.ndarray) -> np.ndarray:
    return (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -52 - 1.0


def gen(code: int, seed: int, rank: int, n: int) -> np.ndarray:
    """n elements of the synthetic stream (identical to ref_harness.cpp gen<T>)."""
    k = np.arange(n, dtype=np.uint64)
    if code in (DOUBLE, FLOAT):
        v = _unif(_draw(seed, rank, k))
        return v.astype(NP[code])
    if code == INT32:
        z = _draw(seed, rank, k)
        return ((z >> np.uint64(33)) % np.uint64(2001)).astype(np.int64).astype(np.int32) - 1000
    re = _unif(_draw(seed, rank, 2 * k))
    im = _unif(_draw(seed, rank, 2 * k + 1))
    if code == CFLOAT:
        out = np.empty(n, np.complex64)
        out.real = re.astype(np.float32)
        out.imag = im.astype(np.float32)
        return out
    return re + 1j * im


_SPECIAL = {np.float64: [np.inf, -np.inf, np.nan, -0.0, 0.0, 1e308, -3.0, 0.5],
            np.float32: [np.inf, -np.inf, np.nan, -0.0, 0.0, 3e38, -3.0, 0.5]}


def add_specials(arr: np.ndarray, code: int, seed: int, rank: int) -> np.ndarray:
    """about one element in 8 gets non-finite / extreme parts (identical to ref_harness.cpp
    add_specials: the rule the 'specials' golden cases were generated with)"""
    if code == INT32:
        return arr
    z = _draw(seed ^ 0x5EC1A1, rank, np.arange(arr.size, dtype=np.uint64))
    hit = (z & np.uint64(7)) == 0
    rt = np.float32 if code in (FLOAT, CFLOAT) else np.float64
    table = np.array(_SPECIAL[rt], rt)
    re = table[((z >> np.uint64(3)) & np.uint64(7)).astype(np.int64)]
    if code in (FLOAT, DOUBLE):
        arr[hit] = re[hit]
    else:
        im = table[((z >> np.uint64(6)) & np.uint64(7)).astype(np.int64)]
        v = arr.view(rt).reshape(-1, 2)
        v[hit, 0] = re[hit]
        v[hit, 1] = im[hit]
    return arr


# ------------------------------------------------------------------ wrappers
def copy_and_transform(code, n_rows, n_cols, src: np.ndarray, src_stride, src_cm,
                       dst: np.ndarray, dst_stride, dst_cm, transpose=False, conjugate=False,
                       alpha=1, beta=0):
    lib().oracle_copy_and_transform(code, n_rows, n_cols, src.ctypes.data, src_stride,
                                    int(src_cm), dst.ctypes.data, dst_stride, int(dst_cm),
                                    int(transpose), int(conjugate), scalar(code, alpha),
                                    scalar(code, beta))


def exec_tile_ops(code, ops: np.ndarray, scalars: np.ndarray, src_base: int = 0,
                  dst_base: int = 0) -> None:
    """Execute a costa_tile_op_t list on host memory, op by op, with the oracle's
    copy_and_transform (the test-side model of one batched kernel launch)."""
    L = lib()
    sc = np.ascontiguousarray(scalars, NP[code]).reshape(-1)
    one, zero = scalar(code, 1), scalar(code, 0)
    for op in ops:
        flags = int(op["flags"])
        kind = (flags >> 4) & 3
        slot = flags >> 16
        if kind == 0:  # BITCOPY ops (pack) ignore the slot scalars
            a, b = one, zero
        else:
            a, b = sc[2 * slot: 2 * slot + 1].tobytes(), sc[2 * slot + 1: 2 * slot + 2].tobytes()
        L.oracle_copy_and_transform(code, int(op["nf"]), int(op["ns"]),
                                    C.c_void_p(src_base + int(op["src"])), int(op["lds"]), 1,
                                    C.c_void_p(dst_base + int(op["dst"])), int(op["ldd"]), 1,
                                    int(flags & 1), int((flags >> 1) & 1), a, b)


def numroc(n, nb, iproc, isrc, nprocs) -> int:
    return lib().oracle_numroc(n, nb, iproc, isrc, nprocs)


def bc_table(m, n, mb, nb, ia, ja, sub_m, sub_n, pm, pn, order, rsrc, csrc, lld, ordering):
    rs = np.zeros(sub_m // mb + 4, np.int32)
    cs = np.zeros(sub_n // nb + 4, np.int32)
    nbr_max = rs.size - 1
    nbc_max = cs.size - 1
    tab = np.zeros(nbr_max * nbc_max * 3, np.int64)
    r = lib().oracle_bc_table(m, n, mb, nb, ia, ja, sub_m, sub_n, pm, pn, order.encode(), rsrc,
                              csrc, lld, ordering.encode(), rs.ctypes.data, cs.ctypes.data,
                              tab.ctypes.data)
    nbr, nbc = int(r // 65536), int(r % 65536)
    return rs[: nbr + 1].copy(), cs[: nbc + 1].copy(), tab[: nbr * nbc * 3].copy()


def transform(code, trans, alpha, beta, A_geom, A_bufs, C_geom, C_bufs):
    """Global oracle: every rank's C buffer updated in place.  *_geom = (rowsplit, colsplit,
    table[nbr*nbc*3] of (owner|-1, element offset, ld), col_major)."""
    ars, acs, atab, acm = A_geom
    crs, ccs, ctab, ccm = C_geom
    ars, acs, crs, ccs = (np.ascontiguousarray(x, np.int32) for x in (ars, acs, crs, ccs))
    atab, ctab = (np.ascontiguousarray(x, np.int64) for x in (atab, ctab))
    ap = (C.c_void_p * len(A_bufs))(*[b.ctypes.data for b in A_bufs])
    cp = (C.c_void_p * len(C_bufs))(*[b.ctypes.data for b in C_bufs])
    rc = lib().oracle_transform(code, trans.encode(), scalar(code, alpha), scalar(code, beta),
                                ars.size - 1, acs.size - 1, ars.ctypes.data, acs.ctypes.data,
                                atab.ctypes.data, int(acm), ap,
                                crs.size - 1, ccs.size - 1, crs.ctypes.data, ccs.ctypes.data,
                                ctab.ctypes.data, int(ccm), cp)
    if rc != 0:
        raise RuntimeError(f"oracle_transform failed ({rc})")


def transform_tiles(code, will_transpose, conj, alpha, beta, src: np.ndarray, dst: np.ndarray,
                    tiles: np.ndarray, nthreads: int = 0) -> None:
    """The reference's CPU tile loop (OpenMP over tiles, 256x256-blocked transpose)."""
    t = np.ascontiguousarray(tiles, np.int64)
    lib().oracle_transform_tiles(code, int(will_transpose), int(conj), scalar(code, alpha),
                                 scalar(code, beta), src.ctypes.data, dst.ctypes.data,
                                 t.ctypes.data, t.shape[0], nthreads)
