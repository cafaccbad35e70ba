"""costa_amd — Python view of the MI355X-native COSTA tile path.

A thin ctypes layer over ``costa_amd/lib/libcosta_amd.so`` (C ABI: include/costa_hip.h).
Names, argument meaning and error behaviour follow the reference's C++ API so tests read
like the reference's own:

    block_cyclic_layout(...)      eth-cscs/COSTA src/costa/layout.hpp:70-86
    custom_layout(...)            src/costa/layout.hpp:34-42
    transform(A, C, comm, ...)    src/costa/grid2grid/transform.hpp:13-43
    transformer(comm)             src/costa/grid2grid/transformer.hpp:8-62
    copy_and_transform(...)       src/costa/grid2grid/memory_utils.hpp:339-412

All compute runs in the HIP library; there is no Python or CPU fallback: a missing or
unloadable library raises ``CostaError`` on first use.

Pointers are plain integers (``tensor.data_ptr()``, ``ndarray.ctypes.data``); they may be
device memory (used in place) or host memory (staged through HBM by the library).
"""
from __future__ import annotations

import ctypes as C
import os
import struct
from dataclasses import dataclass
from typing import Iterable, Sequence

import numpy as np

__all__ = [
    "CostaError", "lib", "FLOAT", "DOUBLE", "CFLOAT", "CDOUBLE", "INT32", "dtype_code",
    "np_dtype", "Layout", "block_cyclic_layout", "custom_layout", "Comm", "transform",
    "transform_batch", "transform_async", "transform_batch_async", "synchronize", "transformer", "copy_and_transform", "execute_tiles", "TileOp",
    "plan_export", "set_profiling", "get_stats", "release_caches", "TILE_OP_DTYPE",
]

FLOAT, DOUBLE, CFLOAT, CDOUBLE, INT32 = 0, 1, 2, 3, 4
_NP = {FLOAT: np.float32, DOUBLE: np.float64, CFLOAT: np.complex64,
       CDOUBLE: np.complex128, INT32: np.int32}

TILE_TRANSPOSE, TILE_CONJ, TILE_VEC_SRC, TILE_VEC_DST = 0x1, 0x2, 0x4, 0x8
SCALE_BITCOPY, SCALE_ZERO, SCALE_ALPHA, SCALE_AXPBY = 0, 1, 2, 3

# numpy view of costa_tile_op_t (40 bytes)
TILE_OP_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("nf", "<i4"), ("ns", "<i4"),
                          ("lds", "<i4"), ("ldd", "<i4"), ("flags", "<u4"),
                          ("order", "<u4")])


class CostaError(RuntimeError):
    """Raised when the native library reports an error (status != COSTA_OK)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[costa status {code}] {msg}")
        self.code = code


def dtype_code(dtype) -> int:
    if isinstance(dtype, int):
        return dtype
    d = np.dtype(dtype)
    for k, v in _NP.items():
        if np.dtype(v) == d:
            return k
    raise ValueError(f"unsupported element type {dtype}")


def np_dtype(code: int):
    return _NP[code]


class _Block(C.Structure):
    _fields_ = [("data", C.c_void_p), ("ld", C.c_int), ("row", C.c_int), ("col", C.c_int)]


_BLOCK_DTYPE = np.dtype([("data", "<u8"), ("ld", "<i4"), ("row", "<i4"), ("col", "<i4")],
                        align=True)
assert _BLOCK_DTYPE.itemsize == C.sizeof(_Block)


class TileOp(C.Structure):
    _fields_ = [("src", C.c_uint64), ("dst", C.c_uint64), ("nf", C.c_int32), ("ns", C.c_int32),
                ("lds", C.c_int32), ("ldd", C.c_int32), ("flags", C.c_uint32),
                ("order", C.c_uint32)]


class PlanInfo(C.Structure):
    _fields_ = [("n_local", C.c_int64), ("n_pack", C.c_int64), ("n_unpack", C.c_int64),
                ("send_elems", C.c_int64), ("recv_elems", C.c_int64),
                ("local_elems", C.c_int64), ("n_ranks", C.c_int32), ("n_slots", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("pack_ms", C.c_double), ("local_ms", C.c_double), ("unpack_ms", C.c_double),
                ("exchange_ms", C.c_double), ("h2d_ms", C.c_double), ("d2h_ms", C.c_double),
                ("pack_launches", C.c_int64), ("local_launches", C.c_int64),
                ("unpack_launches", C.c_int64), ("pack_bytes", C.c_int64),
                ("local_bytes", C.c_int64), ("unpack_bytes", C.c_int64),
                ("transforms", C.c_int64), ("plan_hits", C.c_int64),
                ("plan_misses", C.c_int64), ("host_groups", C.c_int64),
                ("device_plans", C.c_int64), ("plan_ms", C.c_double), ("host_direct", C.c_int64),
                ("host_direct_groups", C.c_int64), ("tile_items", C.c_int64), ("skew_items", C.c_int64),
                ("cblock_items", C.c_int64), ("tiny_items", C.c_int64), ("device_lists", C.c_int64),
                ("fused_pieces", C.c_int64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


# COSTA_LIB: another build of the library (A/B runs against a tuning build of the sources)
LIB_PATH = os.environ.get("COSTA_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                       "lib", "libcosta_amd.so")
_lib = None


def lib():
    """Load libcosta_amd.so (once).  torch is imported first when available so that the
    process holds ONE HIP runtime (torch's libamdhip64 and the system one share a soname)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.environ.get("COSTA_NO_TORCH"):  # COSTA_NO_TORCH=1: the system HIP / RCCL only
        try:                                      # (tests/rccl_system_child.py)
            import torch  # noqa: F401  (see docstring)
        except Exception:  # pragma: no cover - torch absent is fine for pure C users
            pass
    if not os.path.exists(LIB_PATH):
        raise CostaError(-1, f"native library missing: {LIB_PATH} (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    vp, i, c, i64 = C.c_void_p, C.c_int, C.c_char, C.c_int64
    sig = {
        "costa_hip_last_error": (C.c_char_p, []),
        "costa_hip_version": (i, []),
        "costa_hip_block_cyclic_layout": (i, [i, i, i, i, i, i, i, i, i, i, i, c, i, i, vp, i, c, i,
                                              C.POINTER(vp)]),
        "costa_hip_custom_layout": (i, [i, i, i, C.POINTER(i), C.POINTER(i), C.POINTER(i), i,
                                        C.POINTER(_Block), c, C.POINTER(vp)]),
        "costa_hip_layout_destroy": (None, [vp]),
        "costa_hip_layout_reorder_ranks": (i, [vp, C.POINTER(i), i]),
        "costa_hip_layout_num_blocks": (i, [vp]),
        "costa_hip_layout_block": (i, [vp, i, C.POINTER(i), C.POINTER(i), C.POINTER(i),
                                       C.POINTER(i), C.POINTER(vp), C.POINTER(i)]),
        "costa_hip_comm_self": (i, [i, C.POINTER(vp)]),
        "costa_hip_comm_unique_id": (i, [C.c_char_p]),
        "costa_hip_comm_create": (i, [C.c_char_p, i, i, i, C.POINTER(vp)]),
        "costa_hip_comm_rank": (i, [vp]),
        "costa_hip_comm_size": (i, [vp]),
        "costa_hip_comm_destroy": (None, [vp]),
        "costa_hip_transform": (i, [vp, vp, c, vp, vp, vp]),
        "costa_hip_transform_batch": (i, [i, C.POINTER(vp), C.POINTER(vp), C.c_char_p, vp, vp,
                                          vp]),
        "costa_hip_transform_async": (i, [vp, vp, c, vp, vp, vp, vp]),
        "costa_hip_transform_batch_async": (i, [i, C.POINTER(vp), C.POINTER(vp), C.c_char_p, vp,
                                                vp, vp, vp]),
        "costa_hip_synchronize": (i, [vp]),
        "costa_hip_device_count": (i, [C.POINTER(i)]),
        "costa_hip_rccl_version": (i, [C.POINTER(i)]),
        "costa_hip_copy_and_transform": (i, [i, i, i, vp, i, i, vp, i, i, i, i, vp, vp]),
        "costa_hip_execute_tiles": (i, [i, C.POINTER(TileOp), i64, vp, vp, vp, i, i]),
        "costa_hip_plan_export": (i, [i, C.POINTER(vp), C.POINTER(vp), C.c_char_p, vp, vp, i, i,
                                      C.POINTER(PlanInfo), vp, vp, vp, vp, vp, vp, vp, vp]),
        "costa_hip_set_profiling": (i, [i]),
        "costa_hip_get_stats": (i, [C.POINTER(Stats), i]),
        "costa_hip_release_caches": (i, []),
        "costa_hip_set_host_staging": (i, [i]),
        "costa_hip_set_planner": (i, [i]),
        "costa_hip_plan_export_device": (i, [i, i, C.POINTER(vp), C.POINTER(vp), C.c_char_p, vp, vp,
                                             i, i, C.POINTER(PlanInfo), vp, vp, vp, vp, vp, vp, vp,
                                             vp]),
        "costa_hip_set_list_builder": (i, [i]),
        "costa_hip_work_export": (i, [i, vp, i64, i, i, vp, i64, vp, i64, C.POINTER(i64)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc: int):
    if rc != 0:
        raise CostaError(rc, lib().costa_hip_last_error().decode(errors="replace"))


def _ptr(p) -> int:
    """Accept an int address, a numpy array, or anything with data_ptr() (torch tensor)."""
    if p is None:
        return 0
    if isinstance(p, int):
        return p
    if isinstance(p, np.ndarray):
        return p.ctypes.data
    if hasattr(p, "data_ptr"):
        return p.data_ptr()
    raise TypeError(f"cannot take the address of {type(p)}")


def _scalar_bytes(code: int, x) -> bytes:
    if code == DOUBLE:
        return struct.pack("<d", float(x))
    if code == CDOUBLE:
        z = complex(x)
        return struct.pack("<dd", z.real, z.imag)
    return np.asarray(x, dtype=_NP[code]).reshape(1).tobytes()


def _chr(x: str) -> C.c_char:
    return C.c_char(x.encode()[:1])


# ------------------------------------------------------------------ layouts
@dataclass
class BlockInfo:
    row_start: int
    row_end: int
    col_start: int
    col_end: int
    data: int
    ld: int


class Layout:
    """Handle of a native grid_layout (reference grid_layout.hpp:8-189).  Holds references to
    the Python objects owning the memory so they outlive the layout."""

    def __init__(self, handle: int, dtype: int, keep: Iterable = ()):
        self._h = C.c_void_p(handle)
        self.dtype = dtype
        self._keep = list(keep)

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def num_blocks(self) -> int:
        return lib().costa_hip_layout_num_blocks(self._h)

    def block(self, i: int) -> BlockInfo:
        v = [C.c_int() for _ in range(4)]
        d, ld = C.c_void_p(), C.c_int()
        _check(lib().costa_hip_layout_block(self._h, i, *[C.byref(x) for x in v], C.byref(d),
                                            C.byref(ld)))
        return BlockInfo(v[0].value, v[1].value, v[2].value, v[3].value, d.value or 0, ld.value)

    def reorder_ranks(self, reordering: Sequence[int]):
        """Rank relabelling: owner(i, j) -> reordering[owner(i, j)] (reference
        grid_layout::reorder_ranks, grid_layout.hpp:32-34)."""
        p = np.ascontiguousarray(reordering, dtype=np.int32)
        _check(lib().costa_hip_layout_reorder_ranks(self._h, p.ctypes.data_as(C.POINTER(C.c_int)),
                                                    int(p.size)))

    def close(self):
        if self._h and self._h.value:
            lib().costa_hip_layout_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def block_cyclic_layout(m, n, block_m, block_n, i, j, sub_m, sub_n, p_m, p_n, order, rsrc, csrc,
                        ptr, lld, ordering, rank, dtype=DOUBLE) -> Layout:
    """ScaLAPACK block-cyclic layout of sub(A) (reference layout.hpp:70-86)."""
    code = dtype_code(dtype)
    h = C.c_void_p()
    _check(lib().costa_hip_block_cyclic_layout(code, m, n, block_m, block_n, i, j, sub_m, sub_n,
                                               p_m, p_n, _chr(order), rsrc, csrc,
                                               C.c_void_p(_ptr(ptr)), lld, _chr(ordering), rank,
                                               C.byref(h)))
    return Layout(h.value, code, [ptr])


def custom_layout(rowblocks, colblocks, rowsplit, colsplit, owners, localblocks, ordering,
                  dtype=DOUBLE) -> Layout:
    """Arbitrary grid layout (reference layout.hpp:34-42).  ``localblocks`` is a sequence of
    (data, ld, row, col) with data an address/array/tensor."""
    code = dtype_code(dtype)
    rs = np.ascontiguousarray(rowsplit, dtype=np.int32)
    cs = np.ascontiguousarray(colsplit, dtype=np.int32)
    ow = np.ascontiguousarray(owners, dtype=np.int32).reshape(-1)
    lb = list(localblocks)
    # numpy image of costa_block_t[] (built column-wise: ~100x faster than ctypes structs)
    arr = np.zeros(max(1, len(lb)), _BLOCK_DTYPE)
    if lb:
        arr["data"][:len(lb)] = [_ptr(b[0]) for b in lb]
        rest = np.asarray([b[1:4] for b in lb], dtype=np.int64).reshape(len(lb), 3)
        arr["ld"][:len(lb)] = rest[:, 0]
        arr["row"][:len(lb)] = rest[:, 1]
        arr["col"][:len(lb)] = rest[:, 2]
    h = C.c_void_p()
    ip = C.POINTER(C.c_int)
    _check(lib().costa_hip_custom_layout(code, rowblocks, colblocks, rs.ctypes.data_as(ip),
                                         cs.ctypes.data_as(ip), ow.ctypes.data_as(ip), len(lb),
                                         arr.ctypes.data_as(C.POINTER(_Block)), _chr(ordering),
                                         C.byref(h)))
    return Layout(h.value, code, [b[0] for b in lb])


# ------------------------------------------------------------------ communicators
class Comm:
    """One rank per GPU.  ``Comm.self(device)`` for a single rank; for several ranks one rank
    calls ``Comm.unique_id()``, the caller broadcasts the 128 bytes, and every rank calls
    ``Comm.create(uid, nranks, rank, device)`` (collective)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    @staticmethod
    def self(device: int = 0) -> "Comm":
        h = C.c_void_p()
        _check(lib().costa_hip_comm_self(device, C.byref(h)))
        return Comm(h.value)

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        _check(lib().costa_hip_comm_unique_id(buf))
        return buf.raw

    @staticmethod
    def create(uid: bytes, nranks: int, rank: int, device: int) -> "Comm":
        assert len(uid) == 128
        h = C.c_void_p()
        _check(lib().costa_hip_comm_create(uid, nranks, rank, device, C.byref(h)))
        return Comm(h.value)

    @property
    def handle(self):
        return self._h

    @property
    def rank(self) -> int:
        return lib().costa_hip_comm_rank(self._h)

    @property
    def size(self) -> int:
        return lib().costa_hip_comm_size(self._h)

    def close(self):
        if self._h and self._h.value:
            lib().costa_hip_comm_destroy(self._h)
            self._h = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------ transforms
def transform(A: Layout, Cl: Layout, comm: Comm, trans: str = "N", alpha=1, beta=0):
    """sub(C) = beta*sub(C) + alpha*op(sub(A)) (reference transform.hpp:13-27)."""
    transform_batch([A], [Cl], comm, [trans], [alpha], [beta])


def transform_batch(As: Sequence[Layout], Cs: Sequence[Layout], comm: Comm,
                    trans: Sequence[str] | None = None, alpha=None, beta=None):
    """Several layout pairs in one exchange (reference transform.hpp:38-43)."""
    n = len(As)
    assert n == len(Cs) and n > 0
    code = As[0].dtype
    trans = list(trans) if trans is not None else ["N"] * n
    alpha = list(alpha) if alpha is not None else [1] * n
    beta = list(beta) if beta is not None else [0] * n
    a = (C.c_void_p * n)(*[x.handle.value for x in As])
    c = (C.c_void_p * n)(*[x.handle.value for x in Cs])
    ab = b"".join(_scalar_bytes(code, x) for x in alpha)
    bb = b"".join(_scalar_bytes(code, x) for x in beta)
    _check(lib().costa_hip_transform_batch(n, a, c, "".join(trans).encode(), ab, bb, comm.handle))


def transform_async(A: Layout, Cl: Layout, comm: Comm, trans: str = "N", alpha=1, beta=0,
                    stream=None):
    """Stream-ordered transform (device-resident layouts).  `stream`: a torch stream, a raw
    hipStream_t address, or None; it waits for the result.  See costa_hip_transform_async."""
    transform_batch_async([A], [Cl], comm, [trans], [alpha], [beta], stream)


def transform_batch_async(As, Cs, comm: Comm, trans=None, alpha=None, beta=None, stream=None):
    n = len(As)
    code = As[0].dtype
    trans = list(trans) if trans is not None else ["N"] * n
    alpha = list(alpha) if alpha is not None else [1] * n
    beta = list(beta) if beta is not None else [0] * n
    a = (C.c_void_p * n)(*[x.handle.value for x in As])
    c = (C.c_void_p * n)(*[x.handle.value for x in Cs])
    ab = b"".join(_scalar_bytes(code, x) for x in alpha)
    bb = b"".join(_scalar_bytes(code, x) for x in beta)
    s = getattr(stream, "cuda_stream", stream) or 0
    _check(lib().costa_hip_transform_batch_async(n, a, c, "".join(trans).encode(), ab, bb,
                                                 comm.handle, C.c_void_p(s)))


def synchronize(comm: Comm):
    """Wait for every transform queued on the communicator's device."""
    _check(lib().costa_hip_synchronize(comm.handle))


class transformer:
    """Batches layout pairs into one exchange (reference transformer.hpp:8-62)."""

    def __init__(self, comm: Comm):
        self.comm = comm
        self.clear()

    def schedule(self, A: Layout, Cl: Layout, trans: str | None = None, alpha=None, beta=None):
        self.frm.append(A)
        self.to.append(Cl)
        if trans is not None:
            self.trans.append(trans)
            self.alpha.append(alpha)
            self.beta.append(beta)

    def transform(self):
        if self.alpha and len(self.alpha) != len(self.frm):
            raise ValueError("mix of scaled and unscaled schedule() calls")
        if self.alpha:
            transform_batch(self.frm, self.to, self.comm, self.trans, self.alpha, self.beta)
        else:
            transform_batch(self.frm, self.to, self.comm)
        self.clear()

    def clear(self):
        self.frm, self.to, self.trans, self.alpha, self.beta = [], [], [], [], []


def copy_and_transform(dtype, n_rows, n_cols, src, src_stride, src_col_major, dst, dst_stride,
                       dst_col_major, transpose=False, conjugate=False, alpha=1, beta=0):
    """One tile on device pointers (reference memory_utils.hpp:339-412)."""
    code = dtype_code(dtype)
    _check(lib().costa_hip_copy_and_transform(
        code, n_rows, n_cols, C.c_void_p(_ptr(src)), src_stride, int(bool(src_col_major)),
        C.c_void_p(_ptr(dst)), dst_stride, int(bool(dst_col_major)), int(bool(transpose)),
        int(bool(conjugate)), _scalar_bytes(code, alpha), _scalar_bytes(code, beta)))


def execute_tiles(dtype, ops: np.ndarray, scalars: np.ndarray, src_base=0, dst_base=0,
                  device: int = 0):
    """Run a tile-op list (numpy array of TILE_OP_DTYPE) in one batched launch."""
    code = dtype_code(dtype)
    ops = np.ascontiguousarray(ops, dtype=TILE_OP_DTYPE)
    sc = np.ascontiguousarray(scalars, dtype=_NP[code]).reshape(-1)
    assert sc.size % 2 == 0
    _check(lib().costa_hip_execute_tiles(code, ops.ctypes.data_as(C.POINTER(TileOp)), ops.size,
                                         C.c_void_p(_ptr(src_base)), C.c_void_p(_ptr(dst_base)),
                                         sc.ctypes.data, sc.size // 2, device))


@dataclass
class Plan:
    local_ops: np.ndarray
    pack_ops: np.ndarray
    unpack_ops: np.ndarray
    send_counts: np.ndarray
    send_displs: np.ndarray
    recv_counts: np.ndarray
    recv_displs: np.ndarray
    scalars: np.ndarray
    send_elems: int
    recv_elems: int
    local_elems: int


def plan_export(As: Sequence[Layout], Cs: Sequence[Layout], rank: int, nranks: int,
                trans=None, alpha=None, beta=None, device=None) -> Plan:
    """Tile-op lists of `rank`: by the host planner (never touches a GPU), or with ``device``
    set by the GPU planner of that device (costa_hip_plan_export_device)."""
    n = len(As)
    code = As[0].dtype
    trans = list(trans) if trans is not None else ["N"] * n
    alpha = list(alpha) if alpha is not None else [1] * n
    beta = list(beta) if beta is not None else [0] * n
    a = (C.c_void_p * n)(*[x.handle.value for x in As])
    c = (C.c_void_p * n)(*[x.handle.value for x in Cs])
    ab = b"".join(_scalar_bytes(code, x) for x in alpha)
    bb = b"".join(_scalar_bytes(code, x) for x in beta)
    tb = "".join(trans).encode()
    info = PlanInfo()
    L = lib()
    if device is None:
        export = L.costa_hip_plan_export
    else:
        def export(*args):
            return L.costa_hip_plan_export_device(int(device), *args)
    _check(export(n, a, c, tb, ab, bb, rank, nranks, C.byref(info), None, None,
                  None, None, None, None, None, None))
    lo = np.zeros(info.n_local, TILE_OP_DTYPE)
    po = np.zeros(info.n_pack, TILE_OP_DTYPE)
    uo = np.zeros(info.n_unpack, TILE_OP_DTYPE)
    cnt = [np.zeros(nranks, np.int64) for _ in range(4)]
    sc = np.zeros(2 * info.n_slots, _NP[code])
    _check(export(n, a, c, tb, ab, bb, rank, nranks, C.byref(info),
                  lo.ctypes.data, po.ctypes.data, uo.ctypes.data,
                  *[x.ctypes.data for x in cnt], sc.ctypes.data))
    return Plan(lo, po, uo, *cnt, sc, info.send_elems, info.recv_elems, info.local_elems)


# ------------------------------------------------------------------ measurement
def set_profiling(on: bool = True):
    _check(lib().costa_hip_set_profiling(int(on)))


def get_stats(reset: bool = False) -> dict:
    s = Stats()
    _check(lib().costa_hip_get_stats(C.byref(s), int(reset)))
    return s.as_dict()


def release_caches():
    _check(lib().costa_hip_release_caches())


def set_planner(mode: int):
    """Planner of plan-cache misses: 1 = the GPU for layout pairs of >= 4096 blocks (>= 100000
    before the first GPU plan of the process, which loads the planner's kernels; default),
    0 = always the host, 2 = the GPU wherever it applies (costa_hip_set_planner)."""
    _check(lib().costa_hip_set_planner(int(mode)))


def set_list_builder(mode: int):
    """Builder of the work lists' destination-block groups on a plan-cache miss: 1 = the GPU for
    lists of >= 16384 wavefront ops (default), 0 = always the host, 2 = the GPU wherever they apply
    (costa_hip_set_list_builder)."""
    _check(lib().costa_hip_set_list_builder(int(mode)))


@dataclass
class WorkLists:
    ordered: np.ndarray  # TILE_OP_DTYPE: [shaped ops | groups' headers and ops | wavefront pieces]
    work: np.ndarray     # uint64: sub-tile items, then the groups' header indices
    meta: dict           # the work_split counts (costa_hip_work_export)
    on_gpu: bool         # the GPU built the destination-block groups


_WORK_META = ("n_large", "n_medium", "n_skew", "n_cblock", "cblock_lds", "cb_map", "tiny_first",
              "n_tiny", "n_ordered", "n_work", "on_gpu", "flags")


def work_export(dtype, ops: np.ndarray, kind: str = "local", device=None) -> WorkLists:
    """The executor's work lists of one tile-op list (costa_hip_work_export): built on the host, or
    with ``device`` set with the destination-block groups on that GPU.  No kernel runs."""
    code = dtype_code(dtype)
    ops = np.ascontiguousarray(ops, dtype=TILE_OP_DTYPE)
    k = {"local": 0, "pack": 1, "unpack": 2}[kind]
    dev = -1 if device is None else int(device)
    meta = (C.c_int64 * 12)()
    L = lib()
    _check(L.costa_hip_work_export(code, ops.ctypes.data, ops.size, k, dev, None, 0, None, 0, meta))
    o = np.zeros(meta[8], TILE_OP_DTYPE)
    w = np.zeros(meta[9], np.uint64)
    _check(L.costa_hip_work_export(code, ops.ctypes.data, ops.size, k, dev, o.ctypes.data, o.size,
                                   w.ctypes.data, w.size, meta))
    m = dict(zip(_WORK_META, list(meta)))
    return WorkLists(o, w, m, bool(m["on_gpu"]))


def set_host_staging(mode: int):
    """Host-resident layouts: 1 = pipelined (default), 0 = mirror (costa_hip_set_host_staging)."""
    _check(lib().costa_hip_set_host_staging(int(mode)))


def rccl_version() -> int:
    """ncclGetVersion of the RCCL the exchange runs on in this process (major*10000 + minor*100 +
    patch): torch's bundled librccl when torch was imported first, else /opt/rocm's."""
    v = C.c_int(0)
    _check(lib().costa_hip_rccl_version(C.byref(v)))
    return v.value
