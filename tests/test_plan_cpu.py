"""Planner parity on the CPU (no GPU needed).

The product's planner (costa_amd: layouts -> pack / local / unpack tile-op lists, per-peer
counts and displacements) is exported through the C ABI (costa_hip_plan_export) for every
rank of a golden case; the ops are then executed by the ORACLE's copy_and_transform and the
exchange is simulated by slicing the send buffers.  The resulting C buffers must equal the
reference's outputs bit for bit.  This checks the descriptor semantics the HIP kernels
implement, and the pack order agreement between senders and receivers
(communication_data.cpp:103-164, 191-302).
"""
import numpy as np
import pytest

import oracle
from cases import all_cases
from golden_io import first_mismatch, load, matches


def _layouts(costa, case, rank, bufs):
    As, Cs = [], []
    for k, p in enumerate(case.pairs):
        a, c = bufs[k]
        As.append(case.layout_A(k, rank, a.ctypes.data))
        Cs.append(case.layout_C(k, rank, c.ctypes.data))
    return As, Cs


def run_case_cpu(costa, case):
    P = case.P
    bufs = [[case.inputs(k, r) for k in range(len(case.pairs))] for r in range(P)]
    eff = [case.effective(k) for k in range(len(case.pairs))]
    trans = [e[0] for e in eff]
    alpha = [e[1] for e in eff]
    beta = [e[2] for e in eff]
    plans, keep = [], []
    for r in range(P):
        As, Cs = _layouts(costa, case, r, bufs[r])
        keep.append((As, Cs))
        plans.append(costa.plan_export(As, Cs, r, P, trans, alpha, beta))
    E = np.dtype(oracle.NP[case.dtype]).itemsize
    send = [np.zeros(max(1, p.send_elems), oracle.NP[case.dtype]) for p in plans]
    recv = [np.zeros(max(1, p.recv_elems), oracle.NP[case.dtype]) for p in plans]
    for r, p in enumerate(plans):  # PACK
        oracle.exec_tile_ops(case.dtype, p.pack_ops, p.scalars, 0, send[r].ctypes.data)
        assert p.send_counts[r] == 0 and p.recv_counts[r] == 0  # self goes through LOCAL
        assert p.send_counts.sum() == p.send_elems and p.recv_counts.sum() == p.recv_elems
    for r in range(P):  # EXCHANGE (what ncclSend/ncclRecv move)
        for q in range(P):
            n = plans[r].recv_counts[q]
            assert n == plans[q].send_counts[r]
            d, s = plans[r].recv_displs[q], plans[q].send_displs[r]
            recv[r][d:d + n] = send[q][s:s + n]
    for r, p in enumerate(plans):  # UNPACK + LOCAL
        oracle.exec_tile_ops(case.dtype, p.unpack_ops, p.scalars, recv[r].ctypes.data, 0)
        oracle.exec_tile_ops(case.dtype, p.local_ops, p.scalars, 0, 0)
    return bufs, plans


@pytest.mark.parametrize("case", all_cases(), ids=lambda c: c.name)
def test_plan_matches_reference(costa, case):
    fx = load(case.name)
    bufs, _ = run_case_cpu(costa, case)
    for k in range(len(case.pairs)):
        for r in range(case.P):
            key = f"C{k}_r{r}"
            got = bufs[r][k][1]
            assert matches(fx, key, got), f"{case.name} {key}: " + first_mismatch(fx, key, got)


def test_plan_cfg2_geometry(costa):
    """cfg 2 (pxtran fp64 16384^2, 256^2 blocks, 1 rank): 4096 local transposes, no exchange."""
    n, b = 16384, 256
    A = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, 1 << 40, n, "C", 0)
    Cl = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, 1 << 41, n, "C", 0)
    p = costa.plan_export([A], [Cl], 0, 1, ["T"], [1.0], [0.0])
    assert p.local_ops.size == 4096 and p.pack_ops.size == 0 and p.unpack_ops.size == 0
    assert p.local_elems == n * n
    ops = p.local_ops
    assert (ops["nf"] == b).all() and (ops["ns"] == b).all()
    assert (ops["lds"] == n).all() and (ops["ldd"] == n).all()
    assert ((ops["flags"] & costa.TILE_TRANSPOSE) != 0).all()
    assert (((ops["flags"] >> 4) & 3) == costa.SCALE_ALPHA).all()
    # tile (i, j) of A lands at tile (j, i) of C
    src = (ops["src"].astype(np.int64) - (1 << 40)) // 8
    dst = (ops["dst"].astype(np.int64) - (1 << 41)) // 8
    si, sj = src % n // b, src // n // b
    di, dj = dst % n // b, dst // n // b
    assert (si == dj).all() and (sj == di).all()


def test_plan_64bit_offsets(costa):
    """local matrices beyond 2^31 elements: offsets must not wrap (the reference's int
    offsets do, scalapack_layout.cpp:259-266)."""
    n, b = 65536, 128  # 2x2 grid -> 32768^2 = 2^30 per rank; transposed view strides 2^15
    A = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, 1 << 44, n, "C", 0)
    info = A.block(A.num_blocks() - 1)
    assert info.data - (1 << 44) == ((n - b) * n + (n - b)) * 8


def test_errors_are_reported(costa):
    with pytest.raises(costa.CostaError):
        costa.block_cyclic_layout(10, 10, 0, 2, 1, 1, 10, 10, 1, 1, "R", 0, 0, 1 << 40, 10, "C", 0)
    A = costa.block_cyclic_layout(10, 10, 2, 2, 1, 1, 10, 10, 1, 1, "R", 0, 0, 1 << 40, 10, "C", 0)
    Cl = costa.block_cyclic_layout(12, 10, 2, 2, 1, 1, 12, 10, 1, 1, "R", 0, 0, 1 << 41, 12, "C", 0)
    with pytest.raises(costa.CostaError, match="different sizes"):
        costa.plan_export([A], [Cl], 0, 1)
    with pytest.raises(costa.CostaError, match="outside the communicator"):
        B = costa.block_cyclic_layout(10, 10, 2, 2, 1, 1, 10, 10, 2, 1, "R", 0, 0, 1 << 41, 10, "C", 0)
        costa.plan_export([A], [B], 0, 1)
