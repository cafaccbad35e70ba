"""Named parity cases.  Each is run through the REFERENCE (oracle/_ref/ref_harness under
mpiexec) by make_fixtures.py; the outputs are committed next to this file.

Sources of the named cases (eth-cscs/COSTA):
  example0      examples/example0.cpp:80-177   (block-cyclic 'R' grid -> 'C' grid, 'C' -> 'R' data)
  example1      examples/example1.cpp:66-206   (custom layout -> block-cyclic)
  block_cyclic  miniapps/block_cyclic.cpp:60-128 ('T', defaults 1000x1000, 128x128 blocks, 1x1)
  cfg1          BASELINE.json configs[0]: pxgemr2d_miniapp 1024x1024, 128 blocks, 2x2 -> 2x2
  sweep_*       seeded random sweep over grids x blocks x op x alpha/beta x orderings x dtypes,
                submatrices (ia, ja != 1), rank sources, ld padding, custom irregular grids
  batch_*       transformer<T> with several layout pairs in one exchange (transformer.hpp:8-62)
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from casegen import BC, Case, Custom, Pair  # noqa: E402

S, D, CF, Z = 0, 1, 2, 3


def _named():
    cases = []
    cases.append(Case("example0", D, [Pair(BC(4, 4, 2, 2, pm=2, pn=2, order="R", ord="C"),
                                           BC(4, 4, 2, 2, pm=2, pn=2, order="C", ord="R"),
                                           noscale=True)]))
    cases.append(Case("example1", D, [Pair(Custom([0, 2, 4], [0, 2, 4], [[0, 1], [2, 3]], ord="R"),
                                           BC(4, 4, 2, 2, pm=2, pn=2, order="C", ord="C"),
                                           noscale=True)]))
    cases.append(Case("block_cyclic", D, [Pair(BC(1000, 1000, 128, 128),
                                               BC(1000, 1000, 128, 128), trans="T")]))
    cases.append(Case("cfg1", D, [Pair(BC(1024, 1024, 128, 128, pm=2, pn=2, order="R"),
                                       BC(1024, 1024, 128, 128, pm=2, pn=2, order="R"),
                                       noscale=True)]))
    return cases


def _rand_split(rng, n, lo, hi):
    s = [0]
    while s[-1] < n:
        s.append(min(n, s[-1] + int(rng.integers(lo, hi + 1))))
    return s


def _rand_layout(rng, m, n, P, dims_swap=False):
    """random block-cyclic or custom layout of an m x n matrix over P ranks"""
    kind = rng.choice(["bc", "bc", "sub", "custom"])
    ord_ = str(rng.choice(["C", "R"]))
    if kind in ("bc", "sub"):
        grids = [(a, P // a) for a in range(1, P + 1) if P % a == 0]
        pm, pn = grids[int(rng.integers(len(grids)))]
        mb, nb = int(rng.integers(3, 40)), int(rng.integers(3, 40))
        if kind == "sub":
            ia, ja = int(rng.integers(1, 20)), int(rng.integers(1, 20))
            return BC(m + ia - 1 + int(rng.integers(0, 9)), n + ja - 1 + int(rng.integers(0, 9)),
                      mb, nb, ia, ja, m, n, pm, pn, str(rng.choice(["R", "C"])),
                      int(rng.integers(pm)), int(rng.integers(pn)), ord_, int(rng.integers(0, 4)))
        return BC(m, n, mb, nb, pm=pm, pn=pn, order=str(rng.choice(["R", "C"])), ord=ord_,
                  lld_pad=int(rng.integers(0, 3)))
    rs = _rand_split(rng, m, 1, 40)
    cs = _rand_split(rng, n, 1, 40)
    owners = rng.integers(0, P, size=(len(rs) - 1, len(cs) - 1))
    return Custom(rs, cs, owners, ord=ord_, ld_pad=int(rng.integers(0, 3)), gap=int(rng.integers(0, 3)))


SCALARS = {
    S: [(1, 0), (0.5, 0), (-0.5, 2.0), (0, 0), (1, 1)],
    D: [(1, 0), (0.75, 0), (-0.5, 2.0), (0, 0), (1.0, 1.0)],
    CF: [(1, 0), (0.75 - 0.5j, 0), (0.75 - 0.5j, 1.25 + 0.25j), (0, 0), (1j, -1)],
    Z: [(1, 0), (0.75 - 0.5j, 0), (0.75 - 0.5j, 1.25 + 0.25j), (0, 0), (1j, -1)],
}


def _sweep(n_cases=32, seed=20251015):
    rng = np.random.default_rng(seed)
    cases = []
    for k in range(n_cases):
        dt = int(rng.choice([S, D, CF, Z]))
        P = int(rng.choice([1, 2, 3, 4]))
        trans = str(rng.choice(["N", "T", "C"]))
        al, be = SCALARS[dt][int(rng.integers(len(SCALARS[dt])))]
        m, n = int(rng.integers(1, 90)), int(rng.integers(1, 90))
        A = _rand_layout(rng, *( (n, m) if trans != "N" else (m, n) ), P)
        Cl = _rand_layout(rng, m, n, P)
        cases.append(Case(f"sweep_{k:02d}", dt, [Pair(A, Cl, trans, al, be,
                                                     seedA=0xA000 + k, seedC=0xC000 + k)], P=P))
    # transformer batches: two / three pairs, mixed ops, one exchange
    for k, (dt, P) in enumerate([(D, 2), (Z, 3), (S, 4)]):
        pairs = []
        for q in range(2 + k % 2):
            trans = ["N", "T", "C"][(q + k) % 3]
            al, be = SCALARS[dt][(q + 2 * k) % len(SCALARS[dt])]
            m, n = int(rng.integers(5, 70)), int(rng.integers(5, 70))
            A = _rand_layout(rng, *((n, m) if trans != "N" else (m, n)), P)
            Cl = _rand_layout(rng, m, n, P)
            pairs.append(Pair(A, Cl, trans, al, be, seedA=0xB000 + 16 * k + q,
                              seedC=0xD000 + 16 * k + q))
        cases.append(Case(f"batch_{k}", dt, pairs, P=P))
    # no-scale overload with mismatched orderings (implicit transpose) on 2 ranks
    cases.append(Case("noscale_R_to_C", D, [Pair(BC(37, 53, 8, 5, pm=1, pn=2, ord="R"),
                                                 BC(37, 53, 6, 9, pm=2, pn=1, ord="C"),
                                                 noscale=True)], P=2))
    return cases


def all_cases():
    return _named() + _sweep()


def by_name():
    return {c.name: c for c in all_cases()}
