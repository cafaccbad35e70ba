"""The N > 1 path on the CPU: one process per rank (torch.distributed, gloo, world size 2-8).

Each rank plans its own transform with the product planner (costa_hip_plan_export), packs with
the oracle executor, exchanges the packed segments with all_to_all_single using exactly the
per-peer counts and displacements the RCCL send/recv group uses (engine.cpp), unpacks, and
compares its C buffer with the reference's golden output for that rank.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from cases import all_cases  # noqa: E402

WORLDS = (2, 3, 4, 5, 6, 8)
CASES = {p: [c.name for c in all_cases() if c.P == p] for p in WORLDS}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, names, result_dir):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "tests"), os.path.join(root, "tests", "golden")):
        sys.path.insert(0, p)
    import costa_amd as costa
    import oracle
    from cases import by_name
    from golden_io import load, matches

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bad = []
    for name in names:
        case = by_name()[name]
        dt = oracle.NP[case.dtype]
        E = np.dtype(dt).itemsize
        bufs = [case.inputs(k, rank) for k in range(len(case.pairs))]
        As = [case.layout_A(k, rank, bufs[k][0].ctypes.data) for k in range(len(case.pairs))]
        Cs = [case.layout_C(k, rank, bufs[k][1].ctypes.data) for k in range(len(case.pairs))]
        eff = [case.effective(k) for k in range(len(case.pairs))]
        plan = costa.plan_export(As, Cs, rank, world, [e[0] for e in eff], [e[1] for e in eff],
                                 [e[2] for e in eff])
        send = np.zeros(max(1, plan.send_elems), dt)
        recv = np.zeros(max(1, plan.recv_elems), dt)
        oracle.exec_tile_ops(case.dtype, plan.pack_ops, plan.scalars, 0, send.ctypes.data)
        st = torch.from_numpy(send.view(np.uint8))
        rt = torch.from_numpy(recv.view(np.uint8))
        sc = [int(x) * E for x in plan.send_counts]
        rc = [int(x) * E for x in plan.recv_counts]
        # displacements are the exclusive scans in rank order, as all_to_all_single assumes
        assert (plan.send_displs == np.concatenate([[0], np.cumsum(plan.send_counts)[:-1]])).all()
        assert (plan.recv_displs == np.concatenate([[0], np.cumsum(plan.recv_counts)[:-1]])).all()
        dist.all_to_all_single(rt[:sum(rc)], st[:sum(sc)], rc, sc)
        oracle.exec_tile_ops(case.dtype, plan.unpack_ops, plan.scalars, recv.ctypes.data, 0)
        oracle.exec_tile_ops(case.dtype, plan.local_ops, plan.scalars, 0, 0)
        fx = load(name)
        for k in range(len(case.pairs)):
            if not matches(fx, f"C{k}_r{rank}", bufs[k][1]):
                bad.append(f"{name} C{k}_r{rank}")
    with open(os.path.join(result_dir, f"rank{rank}.txt"), "w") as f:
        f.write("\n".join(bad))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", WORLDS)
def test_ranks_gloo(tmp_path, world):
    """every golden case of `world` ranks (grids 1x2 .. 2x4, remaps, custom grids, batches,
    BASELINE cfg 3 / 4 / 5 geometries, relabelled targets)"""
    names = CASES[world]
    assert names, f"no {world}-rank golden cases"
    mp.spawn(_worker, args=(world, _free_port(), names, str(tmp_path)), nprocs=world, join=True)
    bad = []
    for r in range(world):
        txt = (tmp_path / f"rank{r}.txt").read_text().strip()
        if txt:
            bad += txt.splitlines()
    assert not bad, f"mismatches: {bad}"
