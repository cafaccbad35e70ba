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
  cfg3_*        BASELINE configs[2] geometry scaled down: pxgemr2d fp64 2x2 'R' -> 4x1 'R',
                128^2 blocks, no-scale overload, 4 ranks (also with ia, ja != 1 and rank sources)
  cfg4_*        BASELINE configs[3] geometry: pztranu / pztranc complex<double> on a 2x4 'R' grid,
                128^2 blocks, alpha = 0.75-0.5i, beta = 1.25+0.25i, 8 ranks
  cfg5_*        BASELINE configs[4] geometry: custom layouts, A edges 8-96, C edges 16-160,
                owners uniform over 8 ranks, fp32 'N' (alpha 1, beta 0) and 'T' (-0.5, 2)
  relabel_*     transforms onto rank-relabelled targets: grid_layout::reorder_ranks
                (grid_layout.hpp:32-34) with the permutation optimal_reordering gives, applied as
                README.md:343-362 prescribes
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


def _edges(seed, n, lo, hi):
    r = np.random.default_rng(seed)
    s = [0]
    while s[-1] < n:
        s.append(min(n, s[-1] + int(r.integers(lo, hi + 1))))
    return s


def _baseline_geometries():
    """BASELINE.json configs[2..4] at fixture size, on their own rank counts (4 and 8)."""
    cases = []
    # cfg 3: pxgemr2d = the no-scale overload, 2x2 -> 4x1 row-major grids, ragged last blocks
    cases.append(Case("cfg3_remap", D, [Pair(BC(1000, 1100, 128, 128, pm=2, pn=2, order="R"),
                                             BC(1000, 1100, 128, 128, pm=4, pn=1, order="R"),
                                             noscale=True, seedA=0x3A, seedC=0x3C)]))
    cases.append(Case("cfg3_remap_sub", D, [Pair(
        BC(1100, 1200, 128, 128, 37, 51, 1000, 1100, 2, 2, "R", 1, 0, "C", 3),
        BC(1060, 1130, 128, 128, 11, 5, 1000, 1100, 4, 1, "R", 2, 0, "C", 0),
        noscale=True, seedA=0x3B, seedC=0x3D)]))
    # cfg 4: pztranu ('T') and pztranc ('C'); sub(A) is n x m, sub(C) m x n
    m, n = 1200, 1100
    for op in ("T", "C"):
        cases.append(Case(f"cfg4_{op}", Z, [Pair(BC(n, m, 128, 128, pm=2, pn=4, order="R"),
                                                BC(m, n, 128, 128, pm=2, pn=4, order="R"),
                                                op, 0.75 - 0.5j, 1.25 + 0.25j,
                                                seedA=0x4A, seedC=0x4C)]))
    # cfg 5: irregular custom grids, every block its own owner draw over 8 ranks
    m, n = 2048, 1920
    for op, al, be in (("N", 1.0, 0.0), ("T", -0.5, 2.0)):
        am, an = (n, m) if op == "T" else (m, n)
        ars, acs = _edges(0xC5A1, am, 8, 96), _edges(0xC5A2, an, 8, 96)
        crs, ccs = _edges(0xC5A3, m, 16, 160), _edges(0xC5A4, n, 16, 160)
        ao = np.random.default_rng(0xC5A5).integers(0, 8, (len(ars) - 1, len(acs) - 1))
        co = np.random.default_rng(0xC5A6).integers(0, 8, (len(crs) - 1, len(ccs) - 1))
        cases.append(Case(f"cfg5_{op}", S, [Pair(Custom(ars, acs, ao, ord="C"),
                                                Custom(crs, ccs, co, ord="C"), op, al, be,
                                                seedA=0x5A, seedC=0x5C)], P=8))
    return cases


def _split(n, b):
    return list(range(0, n, b)) + [n]


def _relabelled():
    """Targets relabelled by involutions of the kind optimal_reordering proposes (pairs of ranks
    swapped; relabel_readme uses the reference's own proposal for that geometry,
    tests/golden/relabel.json), and one by a 3-cycle."""
    cases = []
    # README.md:461-470 geometry (2x4 'R' -> 4x2 'C' ranks), scaled to 1000^2 / 100^2 blocks
    cases.append(Case("relabel_readme", D, [Pair(
        BC(1000, 1000, 100, 100, pm=2, pn=4, order="R"), BC(1000, 1000, 100, 100, pm=4, pn=2, order="C"),
        noscale=True, seedA=0x7A, seedC=0x7C, relabel=[0, 1, 2, 6, 4, 5, 3, 7])]))
    # the same grid with ranks permuted: relabelled, every tile stays local
    rs = _split(1000, 50)
    own = (np.arange(len(rs) - 1)[:, None] % 2) * 2 + (np.arange(len(rs) - 1)[None, :] % 2)
    sigma = np.array([2, 0, 3, 1])
    cases.append(Case("relabel_permuted", D, [Pair(
        BC(1000, 1000, 50, 50, pm=2, pn=2, order="R"), Custom(rs, rs, sigma[own], ord="C"),
        "N", 0.75, 0.0, seedA=0x7B, seedC=0x7D, relabel=[2, 3, 0, 1])], P=4))
    # 2x3 -> 6x1 remap, complex<double> with alpha, beta
    cases.append(Case("relabel_remap", Z, [Pair(
        BC(1200, 900, 32, 40, pm=2, pn=3, order="R"), BC(1200, 900, 25, 35, pm=6, pn=1, order="R"),
        "N", 0.75 - 0.5j, 1.25 + 0.25j, seedA=0x7E, seedC=0x7F, relabel=[0, 5, 2, 3, 4, 1])]))
    # irregular custom grids over 5 ranks, complex<float> 'T'
    m, n = 700, 500
    a_rs, a_cs = _edges(0x71, n, 10, 90), _edges(0x72, m, 10, 90)
    c_rs, c_cs = _edges(0x73, m, 20, 120), _edges(0x74, n, 20, 120)
    ao = np.random.default_rng(0x75).integers(0, 5, (len(a_rs) - 1, len(a_cs) - 1))
    co = np.random.default_rng(0x76).integers(0, 5, (len(c_rs) - 1, len(c_cs) - 1))
    # a relabelling that is not its own inverse (a 3-cycle and a fixed point): rank r holds the
    # blocks of base rank relabel^-1[r]
    cases.append(Case("relabel_cycle3", D, [Pair(
        BC(300, 260, 32, 24, pm=2, pn=2, order="R"), BC(260, 300, 20, 28, pm=4, pn=1, order="R"),
        "T", 0.75, -1.5, seedA=0x79, seedC=0x7A, relabel=[1, 2, 0, 3])], P=4))
    cases.append(Case("relabel_custom_T", CF, [Pair(
        Custom(a_rs, a_cs, ao, ord="R"), Custom(c_rs, c_cs, co, ord="C"), "T",
        0.75 - 0.5j, 1.25 + 0.25j, seedA=0x77, seedC=0x78, relabel=[0, 3, 4, 1, 2])], P=5))
    return cases


def special_cases():
    """Non-finite and extreme values (~1 element in 8 of A and C: +-inf, NaN, +-0, 1e308 / 3e38):
    the reference's complex products go through GCC's C99 Annex G recovery (libgcc __muldc3 /
    __mulsc3) when both parts of the naive product are NaN.  Kept apart from all_cases(): NaNs
    GENERATED by arithmetic carry a platform-defined sign (x86: negative, GPU: positive), so the
    GPU comparison of these treats both-NaN as equal; everything else is bit for bit."""
    cases = []
    # 'T' with alpha = 1 (the transposing path multiplies by alpha: (inf+inf i)(1+0i) = inf+inf i)
    cases.append(Case("specials_z_T", Z, [Pair(BC(50, 60, 16, 12, ord="C"), BC(60, 50, 10, 14, ord="C"),
                                               "T", 1, 0, seedA=0x51, seedC=0x52, specials=True)]))
    # 'C' with alpha, beta != 0 over an ordering change (implicit transpose cancels the op's)
    cases.append(Case("specials_z_C", Z, [Pair(BC(50, 60, 16, 12, ord="R"), BC(60, 50, 10, 14, ord="C"),
                                               "C", 0.75 - 0.5j, 1.25 + 0.25j, seedA=0x53, seedC=0x54,
                                               specials=True)]))
    # complex<float> 'N' copy mode with alpha, beta; and huge alpha: the overflow recovery branch
    cases.append(Case("specials_c_N", CF, [Pair(BC(70, 40, 9, 11, ord="C"), BC(70, 40, 13, 8, ord="C"),
                                                "N", 1j, -1, seedA=0x55, seedC=0x56, specials=True)]))
    cases.append(Case("specials_c_big", CF, [Pair(BC(40, 70, 9, 11, ord="C"), BC(70, 40, 13, 8, ord="R"),
                                                  "T", 1e30 + 1e30j, 2e25 - 1e25j, seedA=0x57,
                                                  seedC=0x58, specials=True)]))
    # real types, and two ranks (the arithmetic in UNPACK)
    cases.append(Case("specials_d_T", D, [Pair(BC(60, 50, 16, 12, pm=1, pn=2, ord="C"),
                                               BC(50, 60, 10, 14, pm=2, pn=1, ord="C"), "T", -0.5, 2.0,
                                               seedA=0x59, seedC=0x5A, specials=True)], P=2))
    cases.append(Case("specials_z_2r", Z, [Pair(BC(48, 40, 8, 8, pm=2, pn=1, ord="C"),
                                                BC(40, 48, 8, 8, pm=1, pn=2, ord="C"), "T", 1, 0,
                                                seedA=0x5B, seedC=0x5C, specials=True)], P=2))
    return cases


def all_cases():
    return _named() + _sweep() + _baseline_geometries() + _relabelled()


def by_name():
    return {c.name: c for c in all_cases()}
