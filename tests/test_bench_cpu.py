"""bench.py's host logic on the CPU: the N-rank launch decision, the position-hash data and the
position-dependent correctness checks of the N > 1 entries (checksums could not see
misplaced tiles).

The checks run end to end on 2 and 4 gloo ranks with the product planner and the oracle
executor (as test_multirank_gloo.py): a correct transform passes, one with two tiles swapped
or one rank's result left out fails.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launch_decision():
    env = {}
    assert bench.launch_decision(1, env, ["--gpus", "1"]) == ("self", None)
    how, cmd = bench.launch_decision(4, env, ["--gpus", "4", "--steps", "5"], port=29555)
    assert how == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "5"]
    assert cmd[-5] == os.path.join(ROOT, "bench.py")
    # a rank started by a launcher runs itself; a WORLD_SIZE that disagrees with --gpus is an error
    assert bench.launch_decision(4, {"WORLD_SIZE": "4"}, []) == ("self", None)
    with pytest.raises(SystemExit) as e:
        bench.launch_decision(4, {"WORLD_SIZE": "2"}, [])
    assert e.value.code == 2


def test_run_ranks_relays_json_and_rc():
    code = "import sys; print('noise'); print('{\"value\": 1}'); sys.exit(3)"
    r = subprocess.run([sys.executable, "-c",
                        f"import bench; raise SystemExit(bench.run_ranks([{sys.executable!r}, '-c', {code!r}]))"],
                       cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert r.returncode == 3
    assert r.stdout.strip() == '{"value": 1}'
    assert "noise" in r.stderr


def test_run_ranks_kills_a_hung_child_and_reports():
    """a child that never finishes (an RCCL hang, say): its process group is killed at the budget,
    one JSON error line names the last phase each rank reported, rc 124"""
    code = ("import sys, time, subprocess\n"
            "print('[bench rank 0] phase: build workload pxtran', file=sys.stderr, flush=True)\n"
            "print('[bench rank 1] phase: ncclCommInitRank (RCCL 22606)', file=sys.stderr, flush=True)\n"
            # a grandchild in the same group must die with it
            "subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(600)'])\n"
            "time.sleep(600)\n")
    t0 = __import__("time").time()
    r = subprocess.run([sys.executable, "-c",
                        f"import bench; raise SystemExit(bench.run_ranks([{sys.executable!r}, '-c', "
                        f"{code!r}], budget_s=3.0, n_gpus=2))"],
                       cwd=ROOT, capture_output=True, text=True, timeout=60)
    assert __import__("time").time() - t0 < 40
    assert r.returncode == 124, r.stderr
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["error"] == "timeout" and line["n_gpus"] == 2 and line["value"] is None
    assert line["last_phase"] == {"0": "build workload pxtran",
                                  "1": "ncclCommInitRank (RCCL 22606)"}


def test_run_ranks_forwards_sigterm_to_the_ranks(tmp_path):
    """SIGTERM to the parent (the driver's own timeout): the rank group, which runs in its own
    session, is killed with it -- grandchildren included -- and the parent exits 128 + 15"""
    import signal
    import time
    pidfile = tmp_path / "pids"
    code = ("import os, sys, time, subprocess\n"
            "g = subprocess.Popen([sys.executable, '-c', 'import time; time.sleep(600)'])\n"
            f"open({str(pidfile)!r}, 'w').write(f'{{os.getpid()}} {{g.pid}}')\n"
            "time.sleep(600)\n")
    parent = subprocess.Popen([sys.executable, "-c",
                               f"import bench; raise SystemExit(bench.run_ranks([{sys.executable!r}, '-c', "
                               f"{code!r}], budget_s=300.0, n_gpus=2))"],
                              cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    t0 = time.time()
    while not pidfile.exists() or len(pidfile.read_text().split()) < 2:
        assert time.time() - t0 < 60, "child did not start"
        time.sleep(0.1)
    pids = [int(x) for x in pidfile.read_text().split()]
    parent.send_signal(signal.SIGTERM)
    assert parent.wait(timeout=60) == 128 + signal.SIGTERM
    for pid in pids:  # the rank and its grandchild are gone (reaped or zombie-free)
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.1)
        else:
            os.kill(pid, signal.SIGKILL)
            raise AssertionError(f"process {pid} outlived the parent's SIGTERM")


def test_rank_watchdog_reports_phase_and_exits():
    """the in-rank watchdog (for ranks an outside launcher started): rank 0 prints the error line
    with its last phase and the process exits 124 while the main thread is blocked"""
    code = ("import bench, time\n"
            "bench.phase(0, 'exchange')\n"
            "bench.start_watchdog(0, 2, 1.0)\n"
            "time.sleep(60)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 124
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["error"] == "timeout" and line["last_phase"] == {"0": "exchange"}
    assert "budget exceeded in phase 'exchange'" in r.stderr


def test_watchdog_keeps_the_measured_headline():
    """a hang after the headline was measured (an end-to-end or extra-config phase): the error
    line still carries the headline value"""
    code = ("import bench, time\n"
            "bench._partial_line.update({'value': 123.5, 'ms_per_step': 0.7})\n"
            "bench.phase(0, 'end-to-end from host memory')\n"
            "bench.start_watchdog(0, 8, 1.0)\n"
            "time.sleep(60)\n")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 124
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    # a timed-out run is no measurement: value null, the headline as partial_value
    assert line["value"] is None and line["partial_value"] == 123.5
    assert line["ms_per_step"] == 0.7 and line["n_gpus"] == 8
    assert line["error"] == "timeout" and line["last_phase"] == {"0": "end-to-end from host memory"}


def test_roofline_fracs_per_pass():
    """kernel time <= step time must hold within each pass.  The line carries the
    events pass's frac (kernel duration) beside that pass's own step time, and the value pass's
    frac (step bytes over ms_per_step); r4's driver numbers: kernel 0.6989 ms in a 0.7097 ms
    events-pass step, value pass 0.6971 ms"""
    b = 4 * 2 ** 30
    r = bench.pass_fracs(b, 1, 0.6989, 0.6971, 0.7097)
    assert r["events_pass_ms_per_step"] == 0.7097
    assert 0.6989 <= r["events_pass_ms_per_step"]  # kernels of a step inside that pass's step
    assert r["frac_value_pass"] == round(b / 0.6971e-3 / 1e9 / 8000.0, 4)
    # the value pass's frac never exceeds what its own step time allows
    assert r["frac_value_pass"] * 8000.0 * 1e9 * 0.6971e-3 <= b * 1.0001
    assert bench.pass_fracs(b, 1, 0.7, 0.0, 0.7)["frac_value_pass"] is None


def test_gpus_n_without_gpus_exits_nonzero():
    """no GPU here: the parent counts devices (no GPU initialisation) and refuses"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2, r.stderr
    assert "GPU(s) visible" in r.stderr


def test_pos_values_exact_and_spread():
    i = torch.arange(0, 4096, dtype=torch.int64)
    j = torch.arange(0, 4096, dtype=torch.int64).flip(0)
    for kind, bits in (("f64", 52), ("f32", 23)):
        v = bench.pos_values(i, j, bench.SEED_A, kind)
        a = v.abs().double()
        assert bool(((a >= 1) & (a < 2)).all())
        assert len(set(v.tolist())) > 4000  # distinct per position
        # transposed positions differ (a transpose bug is visible)
        assert bool((bench.pos_values(j, i, bench.SEED_A, kind) != v).any())
    z = bench.pos_values(i, j, bench.SEED_C, "c128")
    assert z.dtype == torch.complex128 and bool((z.real != z.imag).all())


def test_bc_global_matches_oracle_geometry():
    """bc_global(local) agrees with the reference geometry restated by the oracle"""
    import oracle
    M, N, b, pm, pn = 100, 70, 8, 3, 2
    lld = oracle.numroc(M, b, 0, 0, pm)
    rs, cs, tab = oracle.bc_table(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0, lld, "C")
    tab = tab.reshape(len(rs) - 1, len(cs) - 1, 3)
    for bi in range(len(rs) - 1):
        for bj in range(len(cs) - 1):
            owner, off, ld = (int(x) for x in tab[bi, bj])
            pr, pc = owner // pn, owner % pn
            li, lj = off % ld, off // ld  # local position of the block's first element
            gi = bench.bc_global(torch.tensor(li), b, pm, pr)
            gj = bench.bc_global(torch.tensor(lj), b, pn, pc)
            assert (int(gi), int(gj)) == (rs[bi], cs[bj])


def test_arena_global_of():
    rs, cs = [0, 3, 8], [0, 2, 7]
    blocks, off = [], 0
    for i in range(2):
        for j in range(2):
            rows, cols = rs[i + 1] - rs[i], cs[j + 1] - cs[j]
            blocks.append((off, rows, i, j))
            off += (rows * cols + 3) // 4 * 4
    ar = bench.Arena(blocks, rs, cs, off, "cpu")
    ok, gi, gj = ar.global_of(torch.arange(off, dtype=torch.int64))
    want = {}
    for o, rows, i, j in blocks:
        for c in range(cs[j + 1] - cs[j]):
            for r in range(rows):
                want[o + r + c * rows] = (rs[i] + r, cs[j] + c)
    for e in range(off):
        if e in want:
            assert bool(ok[e]) and (int(gi[e]), int(gj[e])) == want[e]
        else:
            assert not bool(ok[e])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, kind, corrupt, out_dir):
    sys.path.insert(0, ROOT)
    import bench as B
    import costa_amd as costa
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, b = 48, 8
    pm, pn = B.grid_for(world)
    pr, pc = rank // pn, rank % pn
    M, N = n * pm, n * pn
    if kind == "pxtran":  # C = A^T, fp64 bit copies
        tdt, code, kk, al, be, op = torch.float64, costa.DOUBLE, "f64", 1.0, 0.0, "T"
    else:  # cfg4-like: c128 'T' with alpha, beta
        tdt, code, kk, al, be, op = (torch.complex128, costa.CDOUBLE, "c128", complex(0.75, -0.5),
                                     complex(1.25, 0.25), "T")
    lr_c, lc_c = N // pm, M // pn  # C = op(A) is N x M on the same rank grid
    A = torch.empty(n * n, dtype=tdt)
    Cm = torch.empty(lr_c * lc_c, dtype=tdt)
    B.fill_bc(A, n, n, b, pm, pr, pn, pc, B.SEED_A, kk, chunk_elems=500)
    if be != 0:
        B.fill_bc(Cm, lr_c, lc_c, b, pm, pr, pn, pc, B.SEED_C, kk)
    else:
        Cm.zero_()
    LA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0, A.data_ptr(), n,
                                   "C", rank, dtype=code)
    LC = costa.block_cyclic_layout(N, M, b, b, 1, 1, N, M, pm, pn, "R", 0, 0, Cm.data_ptr(),
                                   lr_c, "C", rank, dtype=code)
    plan = costa.plan_export([LA], [LC], rank, world, [op], [al], [be])
    dt = oracle.NP[code]
    E = np.dtype(dt).itemsize
    send = np.zeros(max(1, plan.send_elems), dt)
    recv = np.zeros(max(1, plan.recv_elems), dt)
    oracle.exec_tile_ops(code, plan.pack_ops, plan.scalars, 0, send.ctypes.data)
    st, rt = torch.from_numpy(send.view(np.uint8)), torch.from_numpy(recv.view(np.uint8))
    sc = [int(x) * E for x in plan.send_counts]
    rc = [int(x) * E for x in plan.recv_counts]
    dist.all_to_all_single(rt[:sum(rc)], st[:sum(sc)], rc, sc)
    if not (corrupt == "drop" and rank == 1):  # rank 1 receives on every grid here
        oracle.exec_tile_ops(code, plan.unpack_ops, plan.scalars, recv.ctypes.data, 0)
    oracle.exec_tile_ops(code, plan.local_ops, plan.scalars, 0, 0)
    if corrupt == "swap" and rank == 0:  # two b x b tiles of C swapped
        c2 = Cm.view(lc_c, lr_c)  # [col][row]
        t = c2[0:b, 0:b].clone()
        c2[0:b, 0:b] = c2[b:2 * b, b:2 * b]
        c2[b:2 * b, b:2 * b] = t
    g = torch.Generator()
    g.manual_seed(rank)
    bad = B.mismatch_bc(Cm, lr_c, lc_c, b, (pm, pr, pn, pc), lambda i, j: (j, i), g, axpby=be != 0,
                        al=al, be=be, kind=kk, n=4000)
    t = torch.tensor([bad], dtype=torch.int64)
    dist.all_reduce(t)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(str(int(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,kind", [(2, "pxtran"), (4, "pxtran"), (4, "cfg4")])
@pytest.mark.parametrize("corrupt", [None, "swap", "drop"])
def test_position_check_multirank(tmp_path, world, kind, corrupt):
    mp.spawn(_worker, args=(world, _free_port(), kind, corrupt, str(tmp_path)), nprocs=world,
             join=True)
    total = {int((tmp_path / f"r{r}.txt").read_text()) for r in range(world)}
    assert len(total) == 1
    total = total.pop()
    if corrupt is None:
        assert total == 0, f"{total} sampled positions differ on a correct transform"
    else:
        assert total > 0, f"the position check missed a {corrupt} error"


def _e2e_worker(rank, world, port, corrupt, out_dir):
    """bench.py's end-to-end leg at N ranks (host_layouts, e2e_leg, host_c_check) over host
    arrays, the transform executed by the oracle with a gloo exchange at the product planner's
    counts and displacements"""
    sys.path.insert(0, ROOT)
    import bench as B
    import costa_amd as costa
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, b = 48, 8
    pm, pn = B.grid_for(world)
    pr, pc = rank // pn, rank % pn
    M, N = n * pm, n * pn
    ha = np.empty(n * n)
    B.fill_bc(torch.from_numpy(ha), n, n, b, pm, pr, pn, pc, B.SEED_A, "f64", chunk_elems=500)
    hc = np.zeros((N // pm) * (M // pn))
    HA, HC = B.host_layouts(costa, ha, hc, M, N, b, pm, pn, rank)
    calls = [0]

    def call():  # one transform: pack -> all-to-all -> unpack, local
        plan = costa.plan_export([HA], [HC], rank, world, ["T"], [1.0], [0.0])
        send = np.zeros(max(1, plan.send_elems))
        recv = np.zeros(max(1, plan.recv_elems))
        oracle.exec_tile_ops(costa.DOUBLE, plan.pack_ops, plan.scalars, 0, send.ctypes.data)
        st, rt = torch.from_numpy(send.view(np.uint8)), torch.from_numpy(recv.view(np.uint8))
        sc = [int(x) * 8 for x in plan.send_counts]
        rc = [int(x) * 8 for x in plan.recv_counts]
        dist.all_to_all_single(rt[:sum(rc)], st[:sum(sc)], rc, sc)
        if not (corrupt == "drop" and rank == 1):
            oracle.exec_tile_ops(costa.DOUBLE, plan.unpack_ops, plan.scalars, recv.ctypes.data, 0)
        oracle.exec_tile_ops(costa.DOUBLE, plan.local_ops, plan.scalars, 0, 0)
        calls[0] += 1

    def sum_over_ranks(x):
        t = torch.tensor([x], dtype=torch.int64)
        dist.all_reduce(t)
        return int(t.item())

    def max_over_ranks(x):
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    g = torch.Generator()
    g.manual_seed(rank)
    bytes_call = 2.0 * 8 * n * n * world
    gb, ms, ok = B.e2e_leg(call, hc, lambda: B.host_c_check(hc, ha, M, N, b, pm, pn, rank, world, g,
                                                              sum_over_ranks),
                           bytes_call, dist.barrier, max_over_ranks, reps=2)
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(f"{int(ok)} {calls[0]} {gb} {ms}")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("corrupt", [None, "drop"])
def test_e2e_host_leg_multirank(tmp_path, world, corrupt):
    """the N-rank end-to-end code path of bench.py: per-rank host A / C, the transform, the
    position check of the host C summed over ranks, the timed calls' max over ranks"""
    mp.spawn(_e2e_worker, args=(world, _free_port(), corrupt, str(tmp_path)), nprocs=world, join=True)
    res = [(tmp_path / f"r{r}.txt").read_text().split() for r in range(world)]
    oks = {int(x[0]) for x in res}
    assert len(oks) == 1  # every rank reports the same verdict
    assert oks.pop() == (0 if corrupt else 1)
    assert all(int(x[1]) == 3 for x in res)  # checked call + 2 timed
    assert len({(x[2], x[3]) for x in res}) == 1 and float(res[0][2]) > 0  # max over ranks


REF_HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


@pytest.mark.skipif(not os.path.exists(REF_HARNESS) or not os.path.exists(bench.MPIEXEC),
                    reason="oracle/_ref/ref_harness (built where /root/reference exists) or MPICH absent")
@pytest.mark.parametrize("n", [2, 4])
def test_multirank_cpu_baseline_in_the_parent(n, monkeypatch):
    """`bench.py --gpus N` (N > 1) runs the reference's multi-rank path
    (ref_harness bench_mr under mpiexec -n N) in the spawning parent before the ranks start, and
    hands rank 0 numeric reference baselines: the headline's and each extra config's (cfg 3 at
    N = 4).  The rank launch is stubbed; the samples are shortened to 1 s."""
    import argparse
    import functools
    import json
    args = argparse.Namespace(gpus=n, no_cpu_baseline=False, workload="pxtran", extra=None,
                              no_extra=False)
    monkeypatch.setattr(bench, "cpu_baseline_multirank",
                        functools.partial(bench.cpu_baseline_multirank, target_s=1.0))
    monkeypatch.setattr(bench, "host_cpus", lambda: (n, {"cpus_usable": n}))
    seen = {}

    def runner(cmd, budget, gpus):
        assert gpus == n and cmd == ["ranks"]
        seen.update(json.load(open(os.environ[bench.CPU_MR_ENV])))
        return 0
    assert bench.spawn_ranks(["ranks"], args, runner=runner) == 0
    assert bench.CPU_MR_ENV not in os.environ  # the file is the parent's, removed after the run
    keys = {"headline"} | ({"cfg3"} if n == 4 else set())
    assert set(seen) == keys, seen
    for k in keys:
        cb = seen[k]
        assert cb["kind"] == "reference" and cb["ranks"] == n and cb["unit"] == "GB/s"
        assert isinstance(cb["value"], float) and cb["value"] > 0 and cb["cores"] == n
        assert "verified" in cb["sample"] and "MPI_Barrier" in cb["sample"]


def test_extra_entries_carry_their_events_pass_step(monkeypatch):
    """every baseline_configs entry prints the step time of the pass its
    phase (kernel) times come from, so kernel <= step holds on the entry's face"""
    import re
    src = open(os.path.join(ROOT, "bench.py")).read()
    body = src[src.index("def summary(w, r, steps)"):src.index("phase(rank, f\"build workload")]
    assert '"events_pass_ms_per_step": round(r["el_ev"] / steps * 1e3, 4)' in body
    assert re.search(r'"phase_ms_per_step": \{k: round\(r\["st"\]\[k \+ "_ms"\] / steps', body)
    # a synthetic entry as summary() builds it: phase times from the events pass never exceed it
    entry = {"ms_per_step": 8.422, "events_pass_ms_per_step": 8.4601,
             "phase_ms_per_step": {"pack": 0.0, "local": 8.4476, "unpack": 0.0}}
    assert max(entry["phase_ms_per_step"].values()) <= entry["events_pass_ms_per_step"]


def test_entries_name_the_kernels_that_ran():
    """the line's cfg 5 entry carries the kernel names that ran, from the
    library's per-kernel work-item counters (costa_stats_t, r6) over the timed steps"""
    st = {"tile_items": 0, "skew_items": 0, "cblock_items": 80741 * 20, "tiny_items": 2362 * 20}
    assert bench.kernels_ran(st, 20, "float") == {"cblock_kernel<float>": 80741, "tiny_kernel<float>": 2362}
    assert bench.kernels_ran({"tile_items": 4096 * 5}, 5, "double") == {"tile_kernel<double>": 4096}
    # pieces run at the end of the group launch are named as such, not as a tiny_kernel launch
    st["fused_pieces"] = 2362 * 20
    assert bench.kernels_ran(st, 20, "float") == {"cblock_kernel<float>": 80741,
                                                  "cblock_kernel<float> pieces": 2362}
    import costa_amd
    names = [f for f, _ in costa_amd.Stats._fields_]
    assert names[-6:] == ["tile_items", "skew_items", "cblock_items", "tiny_items", "device_lists",
                          "fused_pieces"]
