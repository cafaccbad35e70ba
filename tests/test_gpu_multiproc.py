"""The multi-rank path with one PROCESS per rank and the HIP kernels doing every copy: world
sizes 4, 5, 6 and 8 (BASELINE cfg 3 / 4 / 5 geometries, relabelled targets), all ranks on the
one GPU of the box.

Each rank plans its own transform with the product planner, runs its PACK list on the GPU
(costa_hip_execute_tiles into a device send buffer), exchanges the packages with gloo
all_to_all_single using exactly the per-peer counts and displacements the RCCL send/recv group
uses (engine.cpp), then runs its UNPACK and LOCAL lists on the GPU and compares its C buffer
with the reference's golden output for that rank.  RCCL itself refuses two ranks on one GPU
("Duplicate GPU detected"); its group is exercised by the loopback tests and on the driver's
multi-GPU node.  The emulated-rank tests of test_gpu_parity.py run the same kernels in one
process; this one keeps the ranks' address spaces, plans and buffers apart as a real job does.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from cases import all_cases  # noqa: E402

WORLDS = (4, 5, 6, 8)
CASES = {p: [c.name for c in all_cases()
             if c.P == p and (c.name.startswith(("cfg", "relabel")) or p == 4)] for p in WORLDS}


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

    torch.cuda.set_device(0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bad = []
    for name in names:
        case = by_name()[name]
        dt = oracle.NP[case.dtype]
        E = np.dtype(dt).itemsize
        npairs = len(case.pairs)
        host = [case.inputs(k, rank) for k in range(npairs)]
        bufs = [tuple(torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).copy()).cuda()
                      for x in host[k]) for k in range(npairs)]
        As = [case.layout_A(k, rank, bufs[k][0].data_ptr()) for k in range(npairs)]
        Cs = [case.layout_C(k, rank, bufs[k][1].data_ptr()) for k in range(npairs)]
        eff = [case.effective(k) for k in range(npairs)]
        plan = costa.plan_export(As, Cs, rank, world, [e[0] for e in eff], [e[1] for e in eff],
                                 [e[2] for e in eff])
        send = torch.zeros(max(1, plan.send_elems) * E, dtype=torch.uint8, device="cuda")
        recv = torch.zeros(max(1, plan.recv_elems) * E, dtype=torch.uint8, device="cuda")
        if plan.pack_ops.size:  # PACK on the GPU
            costa.execute_tiles(case.dtype, plan.pack_ops, plan.scalars, 0, send.data_ptr())
        torch.cuda.synchronize()
        sc = [int(x) * E for x in plan.send_counts]
        rc = [int(x) * E for x in plan.recv_counts]
        st, rt = send.cpu(), torch.zeros_like(recv, device="cpu")
        dist.all_to_all_single(rt[:sum(rc)], st[:sum(sc)], rc, sc)  # the exchange
        recv.copy_(rt)
        if plan.unpack_ops.size:  # UNPACK, LOCAL on the GPU
            costa.execute_tiles(case.dtype, plan.unpack_ops, plan.scalars, recv.data_ptr(), 0)
        if plan.local_ops.size:
            costa.execute_tiles(case.dtype, plan.local_ops, plan.scalars, 0, 0)
        torch.cuda.synchronize()
        fx = load(name)
        for k in range(npairs):
            got = bufs[k][1].cpu().numpy().view(dt)
            if not matches(fx, f"C{k}_r{rank}", got):
                bad.append(f"{name} C{k}_r{rank}")
        del As, Cs
    with open(os.path.join(result_dir, f"rank{rank}.txt"), "w") as f:
        f.write("\n".join(bad))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", WORLDS)
def test_ranks_one_process_each(tmp_path, world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    names = CASES[world]
    assert names, f"no {world}-rank golden cases"
    mp.spawn(_worker, args=(world, _free_port(), names, str(tmp_path)), nprocs=world, join=True)
    bad = []
    for r in range(world):
        txt = (tmp_path / f"rank{r}.txt").read_text().strip()
        if txt:
            bad += txt.splitlines()
    assert not bad, f"mismatches: {bad}"
