"""GPU: destination-block groups (engine.cpp cblock_groups -> tile_kernels.hip cblock_kernel), the
path custom layouts whose blocks are their own buffers take (BASELINE cfg 5): one workgroup per
contiguous destination range, 16-byte stores.  Ranges off the 16-byte grid (a `gap` of 1-3
elements after each block), C blocks larger than one group (cut into column bands), ragged A
blocks of 8-60, 'N' and 'T', alpha / beta, fp32 / fp64 / int32 -- against the oracle bit for bit, the
arena's gaps untouched.  The same geometry's groups are checked on the CPU
(tools/work_check.cpp cblock, test_work_lists.py)."""
import numpy as np
import pytest

import oracle
from casegen import Custom

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _splits(rng, n, lo, hi):
    s = [0]
    while s[-1] < n:
        s.append(min(n, s[-1] + int(rng.integers(lo, hi + 1))))
    return s


@pytest.mark.parametrize("dt", [oracle.FLOAT, oracle.DOUBLE, oracle.INT32])
@pytest.mark.parametrize("op,alpha,beta", [("T", 1.0, 0.0), ("T", -0.5, 2.0), ("N", 1.0, 0.0),
                                           ("N", 0.75, -1.25)])
@pytest.mark.parametrize("gap", [0, 1, 3])
def test_cblock_vs_oracle(costa, dt, op, alpha, beta, gap):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if dt == oracle.INT32:  # cblock_kernel<int>: integer scalars, exact products
        alpha, beta = {1.0: 1, -0.5: -3, 0.75: 3}[alpha], {0.0: 0, 2.0: 2, -1.25: -1}[beta]
    rng = np.random.default_rng(100 + gap + 7 * dt)
    m, n = 1500, 1300
    am, an = (n, m) if op == "T" else (m, n)  # A is op(C)'s shape
    def custom(rs, cs):
        return Custom(rs, cs, np.zeros((len(rs) - 1, len(cs) - 1), np.int32), gap=gap)
    A = custom(_splits(rng, am, 8, 60), _splits(rng, an, 8, 60))
    # C blocks up to 220 a side: above one group's budget, cut into column bands
    C = custom(_splits(rng, m, 30, 220), _splits(rng, n, 30, 220))
    a = oracle.gen(dt, 1, 0, A.buf_elems(0, 1))
    c = oracle.gen(dt, 2, 0, C.buf_elems(0, 1))
    expected = c.copy()
    oracle.transform(dt, op, alpha, beta, A.geom(1), [a], C.geom(1), [expected])
    da = torch.from_numpy(a.view(np.uint8).copy()).cuda()
    dc = torch.from_numpy(c.view(np.uint8).copy()).cuda()
    LA = A.make_layout(0, da.data_ptr(), 1, dt)
    LC = C.make_layout(0, dc.data_ptr(), 1, dt)
    costa.transform(LA, LC, costa.Comm.self(0), op, alpha, beta)
    torch.cuda.synchronize()
    got = dc.cpu().numpy().view(oracle.NP[dt])
    assert got.tobytes() == expected.tobytes(), (
        f"{int((got.view(np.uint8) != expected.view(np.uint8)).sum())} bytes differ")
