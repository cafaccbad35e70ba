"""Rank-relabelling cases shared by tests/golden/make_relabel_fixtures.py (which runs the
REFERENCE, oracle/_ref/ref_harness relabel) and tests/test_relabel.py (which runs ours,
tests/relabel/relabel_check.cpp).  A case is written as a spec file:
    P trans
    n_rows_split rows_split...   n_cols_split cols_split...   owners (row-major)   [initial grid]
    (the same for the final grid)"""
import numpy as np


def split(n, b):
    s = [0]
    while s[-1] < n:
        s.append(min(n, s[-1] + b))
    return s


def bc_owners(rs, cs, pm, pn, order):
    """block-cyclic owners; order 'R': rank = prow*pn + pcol, 'C': rank = pcol*pm + prow"""
    i = np.arange(len(rs) - 1)[:, None] % pm
    j = np.arange(len(cs) - 1)[None, :] % pn
    return (i * pn + j) if order == "R" else (j * pm + i)


def grid_text(rs, cs, own):
    return (f"{len(rs)} {' '.join(map(str, rs))}\n{len(cs)} {' '.join(map(str, cs))}\n"
            + " ".join(map(str, np.asarray(own, dtype=np.int64).ravel())) + "\n")


def cases():
    """name -> (P, trans, (rs, cs, owners) initial, (rs, cs, owners) final)"""
    out = {}
    # README.md:461-470 (miniapps/comm_volume.cpp): 100000^2, 100^2 blocks, 2x4 row-major ranks
    # -> 4x2 column-major ranks; published "Comm volume reduction [%] = 33.3333"
    rs = split(100000, 100)
    out["readme"] = (8, "N", (rs, rs, bc_owners(rs, rs, 2, 4, "R")),
                     (rs, rs, bc_owners(rs, rs, 4, 2, "C")))
    # transposed, different blocks and grids
    m, n = 3000, 2000
    ars, acs = split(m, 128), split(n, 96)
    crs, ccs = split(n, 100), split(m, 130)
    out["bc_T"] = (6, "T", (ars, acs, bc_owners(ars, acs, 2, 3, "R")),
                   (crs, ccs, bc_owners(crs, ccs, 3, 2, "C")))
    # 2x3 -> 6x1 remap
    rs2, cs2 = split(2400, 64), split(1800, 80)
    out["bc_remap"] = (6, "N", (rs2, cs2, bc_owners(rs2, cs2, 2, 3, "R")),
                       (split(2400, 50), split(1800, 70),
                        bc_owners(split(2400, 50), split(1800, 70), 6, 1, "R")))
    # the same grid with the ranks permuted: the optimal relabelling keeps everything local
    rs3 = split(1000, 50)
    own = bc_owners(rs3, rs3, 2, 2, "R")
    sigma = np.array([2, 0, 3, 1])
    out["permuted"] = (4, "N", (rs3, rs3, own), (rs3, rs3, sigma[own]))
    # irregular custom grids, random owners
    rng = np.random.default_rng(11)

    def rsplit(n, lo, hi):
        s = [0]
        while s[-1] < n:
            s.append(min(n, s[-1] + int(rng.integers(lo, hi + 1))))
        return s
    a_rs, a_cs, c_rs, c_cs = rsplit(700, 10, 90), rsplit(500, 10, 90), rsplit(700, 20, 120), rsplit(500, 20, 120)
    out["custom"] = (5, "N", (a_rs, a_cs, rng.integers(0, 5, (len(a_rs) - 1, len(a_cs) - 1))),
                     (c_rs, c_cs, rng.integers(0, 5, (len(c_rs) - 1, len(c_cs) - 1))))
    return out


def spec_text(case):
    P, trans, a, c = case
    return f"{P} {trans}\n" + grid_text(*a) + grid_text(*c)
