"""Test-case model shared by the fixture generator, the parity tests and the smoke test.

A case = element type + one or more (A layout, C layout, op, alpha, beta) pairs over P ranks.
Layouts are ScaLAPACK block-cyclic (``BC``) or user-defined grids (``Custom``).  Each case can
  * write the spec read by oracle/ref_harness.cpp (the REFERENCE run, fixture generation),
  * produce every rank's input buffers (splitmix64 stream, oracle.gen),
  * compute the expected outputs with the CPU oracle (oracle.transform),
  * build the product's layouts (costa_amd) on given buffers.
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass, field

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import oracle  # noqa: E402

ESIZE = {0: 4, 1: 8, 2: 8, 3: 16, 4: 4}


def rank_to_grid(rank, pm, pn, order):
    if order.upper() == "C":
        return rank % pm, rank // pm
    return rank // pn, rank % pn


@dataclass
class BC:
    """block_cyclic_layout(m, n, mb, nb, ia, ja, subm, subn, pm, pn, order, rsrc, csrc, ...)"""
    m: int
    n: int
    mb: int
    nb: int
    ia: int = 1
    ja: int = 1
    subm: int | None = None
    subn: int | None = None
    pm: int = 1
    pn: int = 1
    order: str = "R"
    rsrc: int = 0
    csrc: int = 0
    ord: str = "C"
    lld_pad: int = 0

    def __post_init__(self):
        if self.subm is None:
            self.subm = self.m - self.ia + 1
        if self.subn is None:
            self.subn = self.n - self.ja + 1

    @property
    def nranks(self):
        return self.pm * self.pn

    def local_dims(self, rank):
        if rank >= self.pm * self.pn:
            return 0, 0
        pr, pc = rank_to_grid(rank, self.pm, self.pn, self.order)
        return (oracle.numroc(self.m, self.mb, pr, self.rsrc, self.pm),
                oracle.numroc(self.n, self.nb, pc, self.csrc, self.pn))

    def sizes(self, P):
        dims = [self.local_dims(r) for r in range(max(P, self.nranks))]
        fast = max(d[0] if self.ord == "C" else d[1] for d in dims)
        slow = max(d[1] if self.ord == "C" else d[0] for d in dims)
        lld = max(1, fast) + self.lld_pad
        return lld, max(1, lld * slow)

    def buf_elems(self, rank, P):
        return self.sizes(P)[1]

    def spec(self, P):
        lld, be = self.sizes(P)
        return (f"kind bc {self.m} {self.n} {self.mb} {self.nb} {self.ia} {self.ja} {self.subm} "
                f"{self.subn} {self.pm} {self.pn} {self.order} {self.rsrc} {self.csrc} "
                f"{self.ord} {lld} {be}\n")

    def geom(self, P):
        lld, _ = self.sizes(P)
        rs, cs, tab = oracle.bc_table(self.m, self.n, self.mb, self.nb, self.ia, self.ja,
                                      self.subm, self.subn, self.pm, self.pn, self.order,
                                      self.rsrc, self.csrc, lld, self.ord)
        return rs, cs, tab, self.ord == "C"

    def shape(self):
        return self.subm, self.subn

    def make_layout(self, rank, ptr, P, dtype):
        import costa_amd
        lld, _ = self.sizes(P)
        return costa_amd.block_cyclic_layout(self.m, self.n, self.mb, self.nb, self.ia, self.ja,
                                             self.subm, self.subn, self.pm, self.pn, self.order,
                                             self.rsrc, self.csrc, ptr, lld, self.ord, rank,
                                             dtype)


@dataclass
class Custom:
    """custom_layout(rowblocks, colblocks, rowsplit, colsplit, owners, localblocks, ordering);
    every rank stores its blocks one after another (row-major block order) in one buffer,
    block ld = fast extent + ld_pad, plus `gap` unused elements after each block."""
    rowsplit: list
    colsplit: list
    owners: np.ndarray
    ord: str = "C"
    ld_pad: int = 0
    gap: int = 0

    def __post_init__(self):
        self.owners = np.asarray(self.owners, np.int32).reshape(len(self.rowsplit) - 1,
                                                                len(self.colsplit) - 1)

    @property
    def nranks(self):
        return int(self.owners.max()) + 1 if self.owners.size else 1

    def _blocks(self, P):
        """per rank: list of (row, col, offset, ld); per rank buffer size"""
        nbr, nbc = self.owners.shape
        per = [[] for _ in range(P)]
        size = [0] * P
        for i in range(nbr):
            for j in range(nbc):
                r = int(self.owners[i, j])
                rows = self.rowsplit[i + 1] - self.rowsplit[i]
                cols = self.colsplit[j + 1] - self.colsplit[j]
                fast, slow = (rows, cols) if self.ord == "C" else (cols, rows)
                ld = max(1, fast) + self.ld_pad
                per[r].append((i, j, size[r], ld))
                size[r] += ld * max(slow - 1, 0) + fast + self.gap if slow > 0 else self.gap
        return per, [max(1, s) for s in size]

    def buf_elems(self, rank, P):
        return self._blocks(P)[1][rank]

    def spec(self, P):
        per, sizes = self._blocks(P)
        nbr, nbc = self.owners.shape
        s = [f"kind custom {nbr} {nbc}",
             " ".join(map(str, self.rowsplit)), " ".join(map(str, self.colsplit)),
             " ".join(map(str, self.owners.reshape(-1).tolist())), self.ord,
             " ".join(map(str, sizes))]
        for r in range(P):
            s.append(f"{len(per[r])} " + " ".join(f"{i} {j} {o} {ld}" for i, j, o, ld in per[r]))
        return "\n".join(s) + "\n"

    def geom(self, P):
        per, _ = self._blocks(P)
        nbr, nbc = self.owners.shape
        tab = np.full((nbr, nbc, 3), -1, np.int64)
        for r in range(P):
            for i, j, off, ld in per[r]:
                tab[i, j] = (r, off, ld)
        return (np.asarray(self.rowsplit, np.int32), np.asarray(self.colsplit, np.int32),
                tab.reshape(-1), self.ord == "C")

    def shape(self):
        return self.rowsplit[-1], self.colsplit[-1]

    def make_layout(self, rank, ptr, P, dtype):
        import costa_amd
        per, _ = self._blocks(P)
        E = ESIZE[costa_amd.dtype_code(dtype)]
        base = ptr if isinstance(ptr, int) else costa_amd._ptr(ptr)
        blocks = [(base + off * E, ld, i, j) for i, j, off, ld in per[rank]]
        nbr, nbc = self.owners.shape
        L = costa_amd.custom_layout(nbr, nbc, self.rowsplit, self.colsplit, self.owners,
                                    blocks, self.ord, dtype)
        L._keep.append(ptr)
        return L


@dataclass
class Pair:
    A: object
    C: object
    trans: str = "N"
    alpha: complex = 1
    beta: complex = 0
    noscale: bool = False  # use the no-scale overload transform(A, C, comm)
    seedA: int = 0xC057A0
    seedC: int = 0xC057C0
    # rank relabelling of the target layout (README.md:343-362, grid2D.hpp:219-229): the C
    # layout is relabelled by reorder_ranks(relabel), so a cell of base owner o belongs to rank
    # relabel[o] and rank r holds the local blocks of base rank relabel^-1[r] (= relabel[r]
    # for the pair swaps optimal_reordering proposes)
    relabel: list | None = None
    specials: bool = False  # ~1 element in 8 of A and C non-finite or extreme (oracle.add_specials)

    def c_rank(self, rank):
        if self.relabel is None:
            return rank
        return int(np.argsort(np.asarray(self.relabel))[rank])


@dataclass
class Case:
    name: str
    dtype: int
    pairs: list = field(default_factory=list)
    P: int | None = None

    def __post_init__(self):
        if self.P is None:
            self.P = max(max(p.A.nranks, p.C.nranks) for p in self.pairs)

    # ---- reference harness spec
    def spec(self) -> str:
        out = [f"dtype {self.dtype}", f"npairs {len(self.pairs)}"]
        for p in self.pairs:
            a, b = complex(p.alpha), complex(p.beta)
            line = (f"trans {p.trans} alpha {a.real!r} {a.imag!r} beta {b.real!r} {b.imag!r} "
                    f"noscale {int(p.noscale)} seedA {p.seedA} seedC {p.seedC}")
            if p.relabel is not None:
                line += f" relabelC {len(p.relabel)} " + " ".join(map(str, p.relabel))
            if p.specials:
                line += " specials 1"
            out.append(line)
            out.append(p.A.spec(self.P).rstrip("\n"))
            out.append(p.C.spec(self.P).rstrip("\n"))
        return "\n".join(out) + "\n"

    # ---- inputs
    def inputs(self, pair_idx, rank):
        p = self.pairs[pair_idx]
        a = oracle.gen(self.dtype, p.seedA, rank, p.A.buf_elems(rank, self.P))
        c = oracle.gen(self.dtype, p.seedC, rank, p.C.buf_elems(p.c_rank(rank), self.P))
        if p.specials:
            oracle.add_specials(a, self.dtype, p.seedA, rank)
            oracle.add_specials(c, self.dtype, p.seedC, rank)
        return a, c

    # ---- the product's layouts of one rank (the C layout relabelled where the pair says so)
    def layout_A(self, k, rank, ptr):
        return self.pairs[k].A.make_layout(rank, ptr, self.P, self.dtype)

    def layout_C(self, k, rank, ptr):
        p = self.pairs[k]
        L = p.C.make_layout(p.c_rank(rank), ptr, self.P, self.dtype)
        if p.relabel is not None:
            L.reorder_ranks(p.relabel)
        return L

    def geom_C(self, k):
        """oracle geometry of the target; a relabelled cell of owner o lives on rank relabel[o]"""
        p = self.pairs[k]
        rs, cs, tab, cm = p.C.geom(self.P)
        if p.relabel is not None:
            t = np.array(tab, np.int64).reshape(-1, 3)
            own = t[:, 0] >= 0
            t[own, 0] = np.asarray(p.relabel, np.int64)[t[own, 0]]
            tab = t.reshape(-1)
        return rs, cs, tab, cm

    # ---- oracle
    def expected(self):
        """[pair][rank] -> expected C buffer (CPU oracle)."""
        res = []
        for k, p in enumerate(self.pairs):
            A = [self.inputs(k, r)[0] for r in range(self.P)]
            Cb = [self.inputs(k, r)[1] for r in range(self.P)]
            al = 1 if p.noscale else p.alpha
            be = 0 if p.noscale else p.beta
            tr = "N" if p.noscale else p.trans
            oracle.transform(self.dtype, tr, al, be, p.A.geom(self.P), A, self.geom_C(k), Cb)
            res.append(Cb)
        return res

    def effective(self, k):
        p = self.pairs[k]
        if p.noscale:
            return "N", 1, 0
        return p.trans, p.alpha, p.beta
