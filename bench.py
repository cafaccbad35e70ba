#!/usr/bin/env python3
"""Benchmark: device-resident tile pack + transpose + unpack (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (one "step" = one costa::transform over all local tiles, data already in HBM):
  N = 1   BASELINE configs[1]: pxtran fp64 16384 x 16384, 256 x 256 blocks, op 'T',
          alpha = 1, beta = 0, 1 x 1 grid -> 4096 local 256^2 transposes per step.
  N > 1   the same per rank (weak scaling): global (16384*pm) x (16384*pn) fp64 on a pm x pn
          rank grid, C = A^T on the transposed grid; remote tiles go pack -> RCCL -> unpack,
          local tiles are transposed in place (overlapping the exchange).
  extra   BASELINE's multi-GPU configurations on the GPU counts they are quoted on, measured
          after the headline in the same processes and reported under "baseline_configs":
          N = 4: configs[2] pxgemr2d fp64 65536^2, 2x2 -> 4x1, 128^2 blocks ('N', RCCL);
          N = 8: configs[3] pztranu c128 32768^2 on 2x4, alpha, beta != 0, and configs[4]
          custom_layout fp32 16384^2 with owners uniform over the 8 ranks.
Timing: W untimed steps; then barrier + device sync, K steps, device sync + barrier; max over
ranks.  value = algorithmic bytes of all ranks / that time (read + write of every
element moved, + read of C when beta != 0).  Rank 0 prints ONE JSON line.
Launch: with N > 1 and no WORLD_SIZE in the environment, bench.py starts the N ranks itself as a
child `torch.distributed.run` and relays rank 0's line and the exit code (launch_decision).
Correctness: every element's value is a hash of its global position (pos_values); after the
transform each rank compares 100 k random positions of its C with the value that position must
hold (bit for bit; beta*C0 + alpha*op(A) rounded like the reference when beta != 0) and the
mismatch counts are summed over the ranks -> "verified".

roofline: the dominant kernel's algorithmic bytes per launch / its average duration from
HIP events recorded on the stream it runs on (costa_hip_get_stats), against 8 TB/s.  Those
events are recorded in a second pass of the same K steps: in the `value` pass they are off, as
they are in the shipped library (each event pair adds ~11 us to a 0.83 ms cfg 2 step).
cpu_baseline: the REFERENCE's own costa::transform (oracle/_ref/ref_harness, compiled from
/root/reference by oracle/Makefile) on the full cfg 2 matrix with every CPU this process may
use, rank 0 at N = 1; our restatement of its tile loop (oracle/) is reported beside it and
stands in, loudly, when the reference binary is absent.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "GB/s device-resident tile pack+transpose+unpack (fp64), % HBM peak"


def grid_for(n: int):
    pm = int(math.isqrt(n))
    while n % pm:
        pm -= 1
    return pm, n // pm


# ------------------------------------------------------------------ N-rank launch
def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_decision(gpus: int, env, argv, port=None):
    """How this process runs `bench.py --gpus N`.
    -> ("self", None): this process is the bench (N = 1, or a rank started by a launcher);
    -> ("spawn", cmd): start N ranks as a child `torch.distributed.run` (never an exec: the parent
       has not touched the GPU and stays to relay rank 0's line and the exit code).
    Raises SystemExit(2) when a launcher's WORLD_SIZE disagrees with --gpus."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {gpus}", file=sys.stderr)
            raise SystemExit(2)
        return "self", None
    if gpus <= 1:
        return "self", None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port if port else _free_port()}",
           os.path.abspath(__file__)] + list(argv)
    return "spawn", cmd


RUN_BUDGET_S = 540.0  # wall-clock budget of an N-rank child (below the driver's own limit)
_PHASE = re.compile(r"^\[bench rank (\d+)\] phase: (.*?)(?: \(t=[0-9.]+ s\))?$")


def run_ranks(cmd, budget_s: float = RUN_BUDGET_S, n_gpus: int = 0) -> int:
    """Run the N-rank child and relay its output: JSON lines (rank 0's result) to stdout,
    everything else to stderr, as it arrives.  Returns the child's exit code.
    The child runs in its own process group under a wall-clock budget: if it has not finished by
    then (a rank stuck in an RCCL call, say), the whole group is killed (SIGTERM, SIGKILL 10 s
    later), one JSON line with "error": "timeout", n_gpus and the last phase each rank reported
    is printed, and 124 is returned."""
    import signal
    import subprocess
    import threading
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    # the ranks' own watchdog fires first, so that rank 0's error line names its phase
    env.setdefault("COSTA_BENCH_RANK_BUDGET_S", str(max(1.0, budget_s - 30.0)))
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                         env=env, bufsize=1, start_new_session=True)
    last = {}

    def relay():
        for line in p.stdout:
            if line.startswith("{"):
                sys.stdout.write(line)
                sys.stdout.flush()
            else:
                m = _PHASE.match(line.rstrip("\n"))
                if m:
                    last[int(m.group(1))] = m.group(2)
                sys.stderr.write(line)
                sys.stderr.flush()

    def kill_group():
        for sig, grace in ((signal.SIGTERM, 10.0), (signal.SIGKILL, 5.0)):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                break
            try:
                p.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue

    # the child group is its own session, so a signal meant for this process (the driver's
    # timeout, Ctrl-C) does not reach the ranks: pass it on, then exit 128 + signal
    def forward(signum, frame):
        kill_group()
        os._exit(128 + signum)

    prev = {}
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            prev[sig] = signal.signal(sig, forward)
        except ValueError:  # not the main thread: the ranks' own watchdog stays the backstop
            pass
    t = threading.Thread(target=relay, daemon=True)
    t.start()
    try:
        rc = p.wait(timeout=budget_s)
    except subprocess.TimeoutExpired:
        kill_group()
        t.join(timeout=5.0)
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": n_gpus,
                          "error": "timeout", "budget_s": budget_s,
                          "last_phase": {str(k): v for k, v in sorted(last.items())}}),
              flush=True)
        return 124
    finally:
        for sig, h in prev.items():
            signal.signal(sig, h)
    t.join(timeout=5.0)
    return rc


_last_phase = ["start"]
# rank 0's result line as far as it is measured: the watchdog prints it (with the error) when a
# later phase hangs, so a hang after the headline measurement still reports the headline
_partial_line: dict = {}


_T0 = time.time()


def phase(rank: int, msg: str):
    """progress line of one rank (stderr, with the seconds since start), parsed by run_ranks and
    kept for the watchdog"""
    _last_phase[0] = msg
    print(f"[bench rank {rank}] phase: {msg} (t={time.time() - _T0:.1f} s)", file=sys.stderr, flush=True)


def start_watchdog(rank: int, world: int, budget_s: float):
    """A rank of an N-rank run (started by run_ranks or by an outside launcher) that is still
    running after budget_s seconds (a hang inside an RCCL call, say) reports its last phase and
    exits with 124; rank 0 first prints the error JSON line.  The launcher then tears down the
    other ranks.  A daemon timer thread: ctypes calls release the GIL, so it fires while the main
    thread waits inside the library."""
    import threading

    def fire():
        msg = f"watchdog: {budget_s:.0f} s budget exceeded in phase '{_last_phase[0]}'"
        print(f"[bench rank {rank}] {msg}", file=sys.stderr, flush=True)
        if rank == 0:
            line = {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world}
            line.update(_partial_line)
            # a timed-out run is no measurement: value stays null, the headline measured so far
            # goes under partial_value
            line["partial_value"] = line.pop("value", None)
            line["value"] = None
            line.update({"error": "timeout", "budget_s": budget_s,
                         "last_phase": {"0": _last_phase[0]}})
            print(json.dumps(line), flush=True)
        os._exit(124)

    t = threading.Timer(budget_s, fire)
    t.daemon = True
    t.start()
    return t


# ------------------------------------------------------------------ synthetic data
# Every element's value is a hash of its GLOBAL position (row, col) and a seed: uniform on
# +-[1, 2) with a 52-bit (fp64) / 23-bit (fp32) pseudo-random mantissa.  Any rank can then
# compute the value any global element must hold after the transform, so the checks below sample
# positions of the local C and compare bit for bit, without moving data between ranks.
# Integer arithmetic only, below 2^63 at every step, so CPU and GPU agree exactly.
_HP = 2147483647  # 2^31 - 1


def pos_hash(i, j, seed: int):
    """int64 tensors (broadcastable) -> int64 in [0, 2^31)"""
    h = (i * 1000003 + j * 998244353 + (seed % _HP)) % _HP
    h = (h * 48271) % _HP
    h = h ^ (h >> 11)
    return (h * 69621) % _HP


def pos_values(i, j, seed: int, kind: str):
    """the synthetic value of global element (i, j) for element kind 'f64' | 'f32' | 'c128'"""
    import torch
    if kind == "c128":
        return torch.complex(pos_values(i, j, seed, "f64"), pos_values(i, j, seed + 7, "f64"))
    h1 = pos_hash(i, j, seed)
    h2 = pos_hash(i, j, seed + 1)
    sign = 1.0 - 2.0 * (h2 & 1).to(torch.float64)
    if kind == "f64":
        mant = (h1 << 21) + (h2 >> 10)                           # < 2^52
        return (1.0 + mant.to(torch.float64) * 2.0 ** -52) * sign  # exact
    mant = h1 >> 8                                               # < 2^23
    return ((1.0 + mant.to(torch.float64) * 2.0 ** -23) * sign).to(torch.float32)  # exact


def bc_global(local, b: int, p: int, q: int):
    """global index of local row (or column) `local` on process row (column) q of p, block b,
    source process 0 (scalapack_layout.cpp:152-177 for ia = 1)"""
    return (local // b * p + q) * b + local % b


def fill_bc(t, lr: int, lc: int, b: int, pm: int, pr: int, pn: int, pc: int, seed: int,
            kind: str, chunk_elems: int = 1 << 26):
    """fill the column-major lr x lc local matrix `t` (flat, ld = lr) of a block-cyclic layout
    with pos_values of its global positions, a column panel at a time"""
    import torch
    dev = t.device
    gi = bc_global(torch.arange(lr, device=dev, dtype=torch.int64), b, pm, pr)
    cols = max(1, chunk_elems // max(lr, 1))
    for c0 in range(0, lc, cols):
        c1 = min(lc, c0 + cols)
        gj = bc_global(torch.arange(c0, c1, device=dev, dtype=torch.int64), b, pn, pc)
        t[c0 * lr:c1 * lr] = pos_values(gi[None, :], gj[:, None], seed, kind).reshape(-1)


class Arena:
    """a rank's blocks of a custom layout stored one after another (bench cfg 5): maps arena
    element indices to global (row, col)"""

    def __init__(self, blocks, rs, cs, size, device):
        import torch
        self.size = size
        off = [o for o, r, i, j in blocks]
        self.off = torch.tensor(off + [size], dtype=torch.int64, device=device)
        self.rows = torch.tensor([r for o, r, i, j in blocks] + [1], dtype=torch.int64, device=device)
        self.cols = torch.tensor([cs[j + 1] - cs[j] for o, r, i, j in blocks] + [0],
                                 dtype=torch.int64, device=device)
        self.r0 = torch.tensor([rs[i] for o, r, i, j in blocks] + [0], dtype=torch.int64, device=device)
        self.c0 = torch.tensor([cs[j] for o, r, i, j in blocks] + [0], dtype=torch.int64, device=device)

    def global_of(self, e):
        """-> (valid, gi, gj) for arena indices e (int64 tensor)"""
        import torch
        k = torch.searchsorted(self.off, e, right=True) - 1
        o = e - self.off[k]
        r, c = o % self.rows[k], o // self.rows[k]
        return c < self.cols[k], self.r0[k] + r, self.c0[k] + c

    def fill(self, t, seed, kind, chunk=1 << 26):
        import torch
        for e0 in range(0, self.size, chunk):
            e = torch.arange(e0, min(self.size, e0 + chunk), device=t.device, dtype=torch.int64)
            ok, gi, gj = self.global_of(e)
            v = pos_values(gi, gj, seed, kind)
            t[e0:e0 + e.numel()] = torch.where(ok, v, torch.zeros_like(v))


def expected_axpby(al, be, c0, a):
    """beta * c0 + alpha * a with the reference's roundings (no FMA): every product
    and sum is its own torch op; complex products as (ac - bd, ad + bc)"""
    import torch
    if not torch.is_complex(a):
        return (be * c0) + (al * a)
    ar, ai, cr, ci = a.real, a.imag, c0.real, c0.imag
    pr = (be.real * cr) - (be.imag * ci)
    pi = (be.real * ci) + (be.imag * cr)
    qr = (al.real * ar) - (al.imag * ai)
    qi = (al.real * ai) + (al.imag * ar)
    return torch.complex(pr + qr, pi + qi)


def count_mismatch(got, exp) -> int:
    """elements whose bit patterns differ"""
    import torch
    iv = {4: torch.int32, 8: torch.int64}
    if torch.is_complex(got):
        got, exp = torch.view_as_real(got), torch.view_as_real(exp)
    g = got.contiguous().view(iv[got.element_size()])
    e = exp.contiguous().view(iv[exp.element_size()])
    return int((g != e).sum().item())


def measured_traffic(alg_bytes: int):
    """HBM bytes per launch phase of this workload, from the newest committed rocprofv3 PMC
    pass of this same bench command (profiles/<tag>/pmc_*.json, one per workload, written by
    tools/save_profiles.py with the gfx950 FETCH_SIZE correction; matched on the algorithmic
    bytes per launch).  PMC counters cannot be read from inside this process, so they come
    from that separate pass."""
    import glob
    best, best_key = None, None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("bytes_per_launch_alg") == alg_bytes and d.get("hbm_bytes_per_launch_corrected"):
            key = d.get("collected", "")  # ISO date of the pass (r3 on); older files by name order
            if best_key is None or key >= best_key:
                best, best_key = (d["hbm_bytes_per_launch_corrected"], os.path.relpath(p, ROOT)), key
    return best if best else (None, None)


def host_cpus():
    """(threads to use, description): the host CPUs this job may use.  On the GPU pool the
    affinity mask shows the whole 256-CPU machine, but one GPU's job gets a CPU share (its cgroup
    quota; OMP_NUM_THREADS is set to it): 256 OpenMP threads under a 16-CPU quota ran the
    reference at 11 GB/s against ~60 with 16 (profiles/r2/).  Order: the cgroup CPU quota, then
    OMP_NUM_THREADS, then the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = os.cpu_count() or 1
    n, src = aff, "affinity mask"
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n, src = max(1, min(aff, int(int(q) // int(p)))), "cgroup cpu.max quota"
    except Exception:
        omp = os.environ.get("OMP_NUM_THREADS", "")
        if omp.isdigit() and int(omp) > 0:
            n, src = min(aff, int(omp)), "OMP_NUM_THREADS"
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return n, {"cpus_usable": n, "cpus_usable_from": src, "cpus_machine": os.cpu_count(),
               "cpu_model": model}


def cpu_baseline(n=16384, b=256, target_s=10.0):
    """Oracle restatement of the reference tile loop (256x256-blocked transpose, OpenMP over
    tiles) on the full cfg 2 matrix (4096 tiles of 256^2 fp64), repeated for ~target_s s."""
    import numpy as np
    import oracle
    threads, info = host_cpus()
    a = np.random.default_rng(1).standard_normal(n * n)  # col-major, ld n
    c = np.zeros(n * n)
    tiles = []
    for j in range(n // b):
        for i in range(n // b):
            # A tile (i, j) -> C tile (j, i): (src_off, lds, dst_off, ldd, F, S)
            tiles.append((i * b + j * b * n, n, j * b + i * b * n, n, b, b))
    tiles = np.array(tiles, np.int64)
    oracle.transform_tiles(1, 1, 0, 1.0, 0.0, a, c, tiles, threads)  # warm-up, first touch
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.transform_tiles(1, 1, 0, 1.0, 0.0, a, c, tiles, threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= target_s or reps >= 1000:
            break
    ok = np.array_equal(c.reshape(n, n).T, a.reshape(n, n))
    bytes_per = 2 * a.nbytes
    out = {"value": round(bytes_per * reps / el / 1e9, 3), "unit": "GB/s", "cores": threads,
           "kind": "port",
           "sample": f"the full cfg 2 matrix: {len(tiles)} tiles of 256x256 fp64 ('T', alpha=1, "
                     f"beta=0), {reps} passes in {el:.1f} s, oracle/costa_oracle.c "
                     f"oracle_transform_tiles, OpenMP {threads} threads, verified={ok}"}
    out.update(info)
    return out


def cpu_baseline_reference(n=16384, b=256, target_s=10.0):
    """The REFERENCE itself on the host cores: oracle/_ref/ref_harness (eth-cscs/COSTA compiled
    from its own sources by oracle/Makefile; the binary travels with the repo snapshot) runs
    costa::transform 'T' (alpha 1, beta 0) on the full cfg 2 matrix (16384^2 fp64, 256^2 blocks,
    one rank) for ~target_s seconds, timed like the reference's miniapps (pxgemr2d_utils.hpp:
    284-292: wall time around each call).  Started as a child process before this process
    touches the GPU.  None (and a warning on stderr) when the binary is absent."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        print("bench.py: WARNING oracle/_ref/ref_harness is absent (build it with "
              "`make -C oracle ref` where /root/reference exists): cpu_baseline falls back to "
              "kind 'port', our restatement of the reference's tile loop", file=sys.stderr)
        return None
    threads, info = host_cpus()
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    try:
        r = subprocess.run([exe, "bench", str(n), str(n), str(b), str(target_s)],
                           capture_output=True, text=True, timeout=6 * target_s + 180, env=env)
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    except Exception as e:
        print(f"bench.py: WARNING reference CPU baseline failed ({e}); using kind 'port'",
              file=sys.stderr)
        return None
    if r.returncode != 0 or not d.get("verified"):
        print("bench.py: WARNING reference CPU baseline not verified; using kind 'port'",
              file=sys.stderr)
        return None
    out = {"value": round(d["GBps"], 3), "unit": "GB/s", "cores": d["threads"], "kind": "reference",
           "sample": f"the full cfg 2 matrix, {n}x{n} fp64 in {b}x{b} blocks on one rank: the "
                     f"reference's costa::transform 'T' (alpha=1, beta=0; planning included, as "
                     f"every reference call re-plans), {d['reps']} calls in {d['seconds']:.1f} s, "
                     f"OpenMP {d['threads']} threads = every CPU this job may use ({info['cpus_usable_from']}; "
                     f"the host has {info['cpus_machine']}), verified C == A^T"}
    out.update(info)
    return out


def host_layouts(costa, ha, hc, M: int, N: int, b: int, pm: int, pn: int, rank: int):
    """the headline's layouts over host arrays: this rank's local A (M x N on pm x pn, ld = its
    local rows) and C = A^T (N x M on the same grid), column-major"""
    HA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0, ha, M // pm, "C", rank)
    HC = costa.block_cyclic_layout(N, M, b, b, 1, 1, N, M, pm, pn, "R", 0, 0, hc, N // pm, "C", rank)
    return HA, HC


def host_c_check(hc, ha, M: int, N: int, b: int, pm: int, pn: int, rank: int, world: int, gen,
                 sum_over_ranks) -> bool:
    """correctness of an end-to-end leg: one rank compares every element (C == A^T); N ranks
    compare the device legs' position samples of their host C, summed over the ranks"""
    import numpy as np
    import torch
    if world == 1:
        return bool(np.array_equal(hc.reshape(N, M), ha.reshape(N, M).T))
    lr_c, lc_c = N // pm, M // pn
    t = torch.from_numpy(hc)
    if gen.device.type != "cpu":
        t = t.to(gen.device)
    bad = mismatch_bc(t, lr_c, lc_c, b, (pm, rank // pn, pn, rank % pn), lambda i, j: (j, i), gen)
    return sum_over_ranks(bad) == 0


def e2e_leg(call, hc, check, bytes_call: float, barrier, max_over_ranks, reps: int = 3,
            before_timed=None):
    """one host-resident leg of the headline (SURVEY §8d's end-to-end rate): C zeroed, a first
    call (plan, staging allocation) whose result is checked, then `reps` timed calls; the time is
    the max over the ranks -> (GBps_algorithmic, ms_per_call, verified)"""
    hc[:] = 0
    call()
    ok = check()
    if before_timed:
        before_timed()
    barrier()
    t1 = time.perf_counter()
    for _ in range(reps):
        call()
    te = max_over_ranks((time.perf_counter() - t1) / reps)
    return round(bytes_call / te / 1e9, 2), round(te * 1e3, 2), ok


def pass_fracs(bytes_per_launch: float, launches_per_step: float, avg_launch_ms: float,
               ms_per_step: float, events_ms_per_step: float) -> dict:
    """The roofline fraction of each timing pass, so that no figure mixes passes: `frac` (the
    line's roofline.frac) = bytes per launch over the kernel's own average duration, from the
    events pass, beside that pass's step time (the kernels of a step fit inside it);
    `frac_value_pass` = the same step's bytes over ms_per_step, the events-off pass `value` comes
    from (its step time bounds its kernel time from above, so this frac is the lower one)."""
    return {
        "events_pass_ms_per_step": round(events_ms_per_step, 4),
        "frac_value_pass": (round(bytes_per_launch * launches_per_step / (ms_per_step * 1e-3) / 1e9
                                  / HBM_PEAK_GBPS, 4) if ms_per_step > 0 else None),
        "avg_launch_ms_note": (
            "frac and avg_launch_ms: the events pass (events_pass_ms_per_step, the same K steps with "
            "a HIP event pair around every phase; kernel time per step <= that step time); "
            "frac_value_pass: the bytes of a step over ms_per_step, the events-off pass of `value`"),
    }


def copy_ceiling(src, dst, col_bytes: int, reps: int = 20):
    """SURVEY §8(d)'s measured ceiling: what plain device copies of the headline's bytes reach on
    this box, in this process, after the timed region (src -> dst, both device buffers of the
    workload; dst is overwritten).  costa_amd/lib/libcosta_ceiling.so (costa_amd/csrc/
    ceiling.hip): kind 0 hipMemcpyDtoD, kind 1 the strided nt copy of 1 KiB column segments
    (16 columns per 256-thread workgroup, 4 vectors per thread), kind 2 a flat nt copy of 16 KiB
    chunks, kind 3 a flat nt copy of 1 KiB per 64-thread workgroup and kind 4 the strided copy
    with 4 columns per workgroup, both one vector per thread (r4: the fastest copies of these
    bytes, profiles/r4zj/).  Median of `reps` HIP-event-timed repetitions each; bytes counted
    like the transform's (read + write)."""
    import ctypes as C
    import statistics
    lib = C.CDLL(os.path.join(ROOT, "costa_amd", "lib", "libcosta_ceiling.so"))
    f = lib.costa_ceiling_copy_ms
    f.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_int,
                  C.POINTER(C.c_float)]
    nbytes = src.numel() * src.element_size()
    out = {}
    for kind, name in ((0, "hipMemcpyDtoD"), (1, "strided_nt_1KiB_segments"), (2, "flat_nt_16KiB"),
                       (3, "flat_nt_1KiB_per_wave"), (4, "strided_nt_1KiB_segments_1vec")):
        ms = (C.c_float * reps)()
        rc = f(kind, src.data_ptr(), dst.data_ptr(), nbytes, col_bytes, reps, ms)
        if rc != 0:
            out[name] = {"error": rc}
            continue
        med = statistics.median(list(ms))
        out[name] = {"ms": round(med, 4), "GBps": round(2 * nbytes / (med * 1e-3) / 1e9, 1),
                     "min_ms": round(min(ms), 4), "reps": reps}
    return out


def cfg5_splits(n: int = 16384):
    """BASELINE configs[4]'s block edges: A rows / cols uniform in [8, 96] (seeds 0xC5A1 /
    0xC5A2), C rows / cols uniform in [16, 160] (0xC5A3 / 0xC5A4), numpy PCG64 streams"""
    import numpy as np

    def splits(seed, lo, hi):
        r = np.random.default_rng(seed)
        s = [0]
        while s[-1] < n:
            s.append(min(n, s[-1] + int(r.integers(lo, hi + 1))))
        return s
    return (splits(0xC5A1, 8, 96), splits(0xC5A2, 8, 96), splits(0xC5A3, 16, 160),
            splits(0xC5A4, 16, 160))


def cpu_baseline_configs(items, target_s: float = 8.0):
    """The REFERENCE's own OpenMP path beside each BASELINE config the run measures
    (baseline_configs): oracle/_ref/ref_harness bench_cfg3 / bench_c128 / bench_custom on one rank
    with every CPU this job may use -- cfg 3 a 16384^2 fp64 'N' copy slice (128^2 blocks), cfg 4 a
    16384^2 complex<double> 'T' alpha, beta slice (128^2 blocks), cfg 5 the full 16384^2 custom
    layouts ('N' or 'T').  Child processes, started before this process touches the GPU.
    -> {entry key: cpu_baseline dict}; configs the binary cannot run are left out (warning)."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        print("bench.py: WARNING oracle/_ref/ref_harness is absent: no CPU baseline beside the "
              "extra configs", file=sys.stderr)
        return {}
    threads, info = host_cpus()
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    out = {}
    for key, kind, edge in items:
        spec = None
        if kind == "cfg3":
            args = ["bench_cfg3", "16384", "128"]
            sample = "a 16384x16384 fp64 slice of configs[2], 128x128 blocks, op N (no-scale copy)"
        elif kind == "cfg4":
            args = ["bench_c128", "16384", "128"]
            sample = ("a 16384x16384 complex<double> slice of configs[3], 128x128 blocks, op T, "
                      "alpha=(0.75,-0.5) beta=(1.25,0.25); the first call checked every 97th element")
        elif kind == "cfg5":
            op = edge if edge in ("N", "T") else "N"
            fd, spec = tempfile.mkstemp(suffix=".txt")
            with os.fdopen(fd, "w") as f:
                for v in cfg5_splits():
                    f.write(f"{len(v)} " + " ".join(map(str, v)) + "\n")
            args = ["bench_custom", spec, op]
            sample = (f"configs[4]'s full 16384x16384 fp32 custom layouts on one rank, op {op}; the "
                      f"first call checked against the definition on every 7th column")
        else:
            continue
        try:
            r = subprocess.run([exe] + args + [str(target_s)], capture_output=True, text=True,
                               timeout=6 * target_s + 240, env=env)
            d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
            if r.returncode != 0 or not d.get("verified"):
                raise RuntimeError(f"rc {r.returncode}, verified {d.get('verified')}")
        except Exception as e:
            print(f"bench.py: WARNING reference CPU baseline of {key} failed ({e})", file=sys.stderr)
            continue
        finally:
            if spec:
                os.unlink(spec)
        out[key] = {"value": round(d["GBps"], 3), "unit": "GB/s", "cores": d["threads"],
                    "kind": "reference",
                    "sample": f"{sample}: the reference's costa::transform (planning included, as "
                              f"every reference call re-plans), {d['reps']} calls in "
                              f"{d['seconds']:.1f} s, OpenMP {d['threads']} threads, verified"}
    return out


CPU_MR_ENV = "COSTA_BENCH_CPU_MR"
MPIEXEC = "/opt/conda/bin/mpiexec"  # MPICH, the MPI the reference harness is linked against


def cpu_baseline_multirank(world: int, keys_x, target_s: float = 6.0, exe=None):
    """The REFERENCE's multi-rank path beside an N-rank line (N = world): oracle/_ref/ref_harness
    bench_mr under `mpiexec -n N` on the host cores -- every rank packs, exchanges by MPI
    Isend / Irecv and unpacks (transform.cpp:46-128), each call between two MPI_Barriers
    (utils/pxgemr2d_utils.hpp:284-292).  The usable CPUs are split over the ranks (OpenMP threads
    per rank).  Workloads, shrunk to slices the host holds and runs in seconds:
      headline  pxtran fp64 'T' weak-scaled, 8192^2 per rank (the GPU line: 16384^2) on the
                same pm x pn grid, 256^2 blocks
      cfg3      pxgemr2d fp64 'N' 2x2 -> 4x1 remap (N = 4), 8192^2 per rank (16384^2 global;
                the GPU line: 65536^2), 128^2 blocks
      cfg4      pztranu c128 'T' alpha, beta on 2x4 (N = 8), 16384^2 global (GPU: 32768^2)
      cfg5      the full 16384^2 fp32 custom layouts, owners uniform over the N ranks ('N'/'T')
    Child processes only, started before anything touches the GPU.
    -> {"headline" | entry key: cpu_baseline dict (kind "reference", ranks N)}; a workload the
    binary cannot run is left out with a warning on stderr."""
    import shutil
    import subprocess
    import tempfile
    import numpy as np
    exe = exe or os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    mpiexec = MPIEXEC if os.path.exists(MPIEXEC) else shutil.which("mpiexec")
    if not os.path.exists(exe) or not mpiexec:
        print("bench.py: WARNING oracle/_ref/ref_harness or mpiexec absent: no multi-rank CPU "
              "baseline", file=sys.stderr)
        return {}
    threads, info = host_cpus()
    per = max(1, threads // world)
    pm, pn = grid_for(world)
    env = dict(os.environ, OMP_NUM_THREADS=str(per))
    env["PATH"] = os.path.dirname(mpiexec) + ":" + env.get("PATH", "")
    out = {}
    for key, kind, edge in [("headline", "pxtran", None)] + list(keys_x):
        spec = None
        if kind == "pxtran":
            args = ["pxtran", "8192", "256", str(pm), str(pn)]
            sample = (f"pxtran fp64 'T' alpha=1 beta=0 weak-scaled, {8192 * pm}x{8192 * pn} on the "
                      f"{pm}x{pn} rank grid (8192^2 per rank: a quarter of the GPU line's), 256x256 "
                      f"blocks")
        elif kind == "cfg3":
            cm = world  # C on world x 1
            args = ["cfg3", "8192", "128", str(pm), str(pn)]
            sample = (f"pxgemr2d fp64 'N' {8192 * pm}x{8192 * pn}, {pm}x{pn} -> {cm}x1 remap, "
                      f"128x128 blocks (a slice of configs[2]'s 65536^2)")
        elif kind == "cfg4":
            args = ["cfg4", "16384", "128", str(pm), str(pn)]
            sample = (f"pztranu complex<double> 'T' alpha=(0.75,-0.5) beta=(1.25,0.25), 16384x16384 "
                      f"on the {pm}x{pn} rank grid, 128x128 blocks (a slice of configs[3]'s 32768^2)")
        elif kind == "cfg5":
            op = edge if edge in ("N", "T") else "N"
            fd, spec = tempfile.mkstemp(suffix=".txt")
            ars, acs, crs, ccs = cfg5_splits()
            aown = np.random.default_rng(0xC5A5).integers(0, world, (len(ars) - 1, len(acs) - 1))
            cown = np.random.default_rng(0xC5A6).integers(0, world, (len(crs) - 1, len(ccs) - 1))
            with os.fdopen(fd, "w") as f:
                for rs, cs, own in ((ars, acs, aown), (crs, ccs, cown)):
                    f.write(f"{len(rs)} " + " ".join(map(str, rs)) + "\n")
                    f.write(f"{len(cs)} " + " ".join(map(str, cs)) + "\n")
                    f.write(" ".join(map(str, own.reshape(-1).tolist())) + "\n")
            args = ["custom", spec, op]
            sample = (f"configs[4]'s full 16384x16384 fp32 custom layouts, owners uniform over the "
                      f"{world} ranks (as the GPU line), op {op}")
        else:
            continue
        try:
            r = subprocess.run([mpiexec, "-n", str(world), exe, "bench_mr"] + args + [str(target_s)],
                               capture_output=True, text=True, timeout=8 * target_s + 120, env=env)
            d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
            if r.returncode != 0 or not d.get("verified"):
                raise RuntimeError(f"rc {r.returncode}, verified {d.get('verified')}")
        except Exception as e:
            print(f"bench.py: WARNING multi-rank reference CPU baseline of {key} failed ({e})",
                  file=sys.stderr)
            continue
        finally:
            if spec:
                os.unlink(spec)
        out[key] = {"value": round(d["GBps"], 3), "unit": "GB/s", "cores": d["threads"] * d["ranks"],
                    "kind": "reference", "ranks": d["ranks"],
                    "sample": f"{sample}: the reference's costa::transform on {d['ranks']} MPI ranks "
                              f"(MPICH, one host; planning included, as every reference call "
                              f"re-plans), each call between two MPI_Barriers, {d['reps']} calls in "
                              f"{d['seconds']:.1f} s, OpenMP {d['threads']} threads a rank, verified"}
        out[key].update(info)
    return out


def cfg5_workload(costa, torch, rank, world, op):
    """BASELINE configs[4]: fp32 16384^2 custom_layout; A tile edges uniform in
    [8, 96] (seeds 0xC5A1 rows / 0xC5A2 cols), C edges uniform in [16, 160] (0xC5A3 / 0xC5A4),
    owners uniform over the ranks (0xC5A5 for A, 0xC5A6 for C); every owned block is its own
    column-major buffer (ld = rows) in a 256-byte-aligned arena.  numpy PCG64 streams are used
    for the draws.  op 'N' alpha=1 beta=0, or the 'T' variant alpha=-0.5 beta=2."""
    import numpy as np
    ars, acs, crs, ccs = cfg5_splits()
    aown = np.random.default_rng(0xC5A5).integers(0, world, (len(ars) - 1, len(acs) - 1))
    cown = np.random.default_rng(0xC5A6).integers(0, world, (len(crs) - 1, len(ccs) - 1))

    def arena(rs, cs, own):
        blocks, off = [], 0
        for i in range(len(rs) - 1):
            for j in range(len(cs) - 1):
                if own[i, j] != rank:
                    continue
                rows, cols = rs[i + 1] - rs[i], cs[j + 1] - cs[j]
                blocks.append((off, rows, i, j))
                off += (rows * cols + 63) // 64 * 64  # 256-byte aligned blocks
        return blocks, max(off, 64)

    ab, an = arena(ars, acs, aown)
    cb, cn = arena(crs, ccs, cown)
    aa = Arena(ab, ars, acs, an, "cuda")
    ca = Arena(cb, crs, ccs, cn, "cuda")
    A = torch.empty(an, dtype=torch.float32, device="cuda")
    C = torch.empty(cn, dtype=torch.float32, device="cuda")
    aa.fill(A, SEED_A, "f32")
    ca.fill(C, SEED_C, "f32")
    pa, pc = A.data_ptr(), C.data_ptr()
    LA = costa.custom_layout(len(ars) - 1, len(acs) - 1, ars, acs, aown,
                             [(pa + 4 * o, r, i, j) for o, r, i, j in ab], "C", costa.FLOAT)
    LC = costa.custom_layout(len(crs) - 1, len(ccs) - 1, crs, ccs, cown,
                             [(pc + 4 * o, r, i, j) for o, r, i, j in cb], "C", costa.FLOAT)
    al, be = (1.0, 0.0) if op == "N" else (-0.5, 2.0)
    wl = (f"costa::custom_layout fp32 16384x16384, irregular tiles (A edges 8-96: "
          f"{len(ars) - 1}x{len(acs) - 1} blocks, C edges 16-160: {len(crs) - 1}x{len(ccs) - 1}), "
          f"owners uniform over {world} rank(s), op {op} (BASELINE configs[4])")

    def mask(blocks, cs, size):  # the elements the blocks cover (not the arena padding)
        m = np.zeros(size + 1, np.int32)
        for o, r, i, j in blocks:
            m[o] += 1
            m[o + r * (cs[j + 1] - cs[j])] -= 1
        return torch.from_numpy(np.cumsum(m[:size]) > 0).cuda()
    masks = (mask(ab, acs, an), mask(cb, ccs, cn))
    return LA, LC, A, C, op, al, be, wl, masks, ca


SEED_A, SEED_C = 0xC057A0, 0xC057C0  # SURVEY §8d's seeds, here keys of the position hash
N_SAMPLES = 100_000


def mismatch_bc(Cm, lr_c, lc_c, b, cgrid, a_of, gen, axpby=False, al=1.0, be=0.0, kind="f64",
                n=None):
    """position check of a block-cyclic target (source process 0, 'C' storage, ld = lr_c): n
    random local elements of C against the value their global position must hold, bit for bit
    -> the number that differ.  cgrid = (p_rows, my_row, p_cols, my_col) of C's rank grid;
    a_of(gi, gj) -> the (row, col) of A the element comes from; axpby: C held pos_values(SEED_C)
    before the call, expect beta*C0 + alpha*A"""
    import torch
    pm_c, pr_c, pn_c, pc_c = cgrid
    k = torch.randint(0, lr_c * lc_c, (n or N_SAMPLES,), device=Cm.device, generator=gen)
    gi = bc_global(k % lr_c, b, pm_c, pr_c)
    gj = bc_global(k // lr_c, b, pn_c, pc_c)
    ai, aj = a_of(gi, gj)
    exp = pos_values(ai, aj, SEED_A, kind)
    if axpby:
        exp = expected_axpby(al, be, pos_values(gi, gj, SEED_C, kind), exp)
    return count_mismatch(Cm[k], exp)


def mismatch_arena(Cm, ca, op, gen, C0=None, al=1.0, be=0.0, n=None):
    """the same for a custom-layout arena (bench cfg 5, fp32): positions of the local C arena
    (padding skipped); C0: C before the call when beta != 0"""
    import torch
    n = n or N_SAMPLES
    e = torch.randint(0, ca.size, (2 * n,), device=Cm.device, generator=gen)
    ok, gi, gj = ca.global_of(e)
    e, gi, gj = e[ok][:n], gi[ok][:n], gj[ok][:n]
    ai, aj = (gi, gj) if op == "N" else (gj, gi)
    exp = pos_values(ai, aj, SEED_A, "f32")
    if C0 is not None:
        exp = expected_axpby(al, be, C0[e], exp)
    return count_mismatch(Cm[e], exp)


def kernels_ran(st: dict, steps: int, tname: str) -> dict:
    """the kernels a step launched and their work items per step, from the library's counters
    (costa_stats_t tile_items / skew_items / cblock_items / tiny_items): tile_kernel sub-tiles,
    skew_kernel sub-tiles, cblock_kernel destination-block groups, tiny_kernel wavefront pieces"""
    out = {}
    fused = st.get("fused_pieces", 0)  # pieces run in the group kernel's launch (its tail)
    counts = {"tile_items": st.get("tile_items", 0), "skew_items": st.get("skew_items", 0),
              "cblock_items": st.get("cblock_items", 0), "tiny_items": st.get("tiny_items", 0) - fused,
              "fused_pieces": fused}
    for key, name in (("tile_items", "tile_kernel"), ("skew_items", "skew_kernel"),
                      ("cblock_items", "cblock_kernel"), ("tiny_items", "tiny_kernel"),
                      ("fused_pieces", "cblock_kernel pieces")):
        n = counts[key] / max(steps, 1)
        if n:
            label = f"cblock_kernel<{tname}> pieces" if key == "fused_pieces" else f"{name}<{tname}>"
            out[label] = int(n) if float(n).is_integer() else round(n, 1)
    return out


def extra_keys(world: int, args):
    """BASELINE's other configurations, measured after the headline in the same processes: at
    the GPU counts they are quoted on (cfg 3 at 4 GPUs, cfg 4 and cfg 5 at 8), and at one GPU
    their single-GPU slices, each beside the reference's own CPU rate.
    -> [(entry key, config, edge / op)]"""
    extra_plan = {1: [("cfg3", None), ("cfg4", 32768), ("cfg5", "N"), ("cfg5", "T")],
                  4: [("cfg3", None)], 8: [("cfg4", 32768), ("cfg5", "N")]}
    plan_x = extra_plan.get(world, [])
    if args.extra:
        plan_x = []
        for item in args.extra.split(","):
            k, _, e = item.partition(":")
            plan_x.append((k, (int(e) if e.isdigit() else e) if e else None))
    if args.workload != "pxtran" or args.no_extra:
        plan_x = []
    keys_x = []
    for kind, edge in plan_x:
        used = {k for k, _, _ in keys_x}
        keys_x.append((kind if kind not in used else f"{kind}_{edge}", kind, edge))
    return keys_x


def spawn_ranks(cmd, args, runner=None) -> int:
    """The parent of `bench.py --gpus N` (N > 1, no launcher): the reference's multi-rank CPU
    baselines first (cpu_baseline_multirank, before any rank touches the GPU; their results reach
    rank 0 through a file named by COSTA_BENCH_CPU_MR), then the N ranks (run_ranks, or `runner`
    in the tests) -> the ranks' exit code"""
    import tempfile
    runner = runner or run_ranks
    budget = float(os.environ.get("COSTA_BENCH_BUDGET_S", RUN_BUDGET_S))
    path = None
    if not args.no_cpu_baseline and args.workload == "pxtran":
        mr = cpu_baseline_multirank(args.gpus, extra_keys(args.gpus, args))
        fd, path = tempfile.mkstemp(prefix="costa_cpu_mr_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(mr, f)
        os.environ[CPU_MR_ENV] = path
    try:
        return runner(cmd, budget, args.gpus)
    finally:
        if path:
            os.environ.pop(CPU_MR_ENV, None)
            os.unlink(path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--edge", type=int, default=16384, help="local matrix edge per rank")
    ap.add_argument("--block", type=int, default=256)
    ap.add_argument("--workload", choices=["pxtran", "cfg3", "cfg4", "cfg5"], default="pxtran",
                    help="pxtran: BASELINE configs[1] (default, the headline); cfg3: configs[2] "
                         "pxgemr2d fp64 remap pm x pn -> world x 1, 128^2 blocks, 32768^2 per "
                         "rank (65536^2 2x2 -> 4x1 at 4 ranks); cfg4: configs[3] "
                         "pztranu c128 alpha,beta != 0, 128^2 blocks (16384^2 per rank); cfg5: "
                         "configs[4] custom_layout many-small fp32 tiles")
    ap.add_argument("--cfg5-op", choices=["N", "T"], default="N")
    ap.add_argument("--cfg4-beta0", action="store_true",
                    help="cfg4 with beta = 0 (A/B of the third stream; not a BASELINE config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip BASELINE's multi-GPU configs (cfg 3 at 4 GPUs, cfg 4 / 5 at 8)")
    ap.add_argument("--extra", default=None,
                    help="run these extra configs instead of the GPU count's own, e.g. "
                         "'cfg3,cfg4:32768,cfg5:N' (rehearsal of the multi-GPU entries)")
    args = ap.parse_args()

    # `bench.py --gpus N` with N > 1 and no launcher around it: start the N ranks as a child
    # torch.distributed.run (before anything here touches the GPU), relay rank 0's line
    how, cmd = launch_decision(args.gpus, os.environ, sys.argv[1:])
    if how == "spawn":
        import torch
        have = torch.cuda.device_count()  # counts devices without initialising the GPU
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but {have} GPU(s) visible", file=sys.stderr)
            raise SystemExit(2)
        raise SystemExit(spawn_ranks(cmd, args))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "pxtran"
    keys_x = extra_keys(world, args)
    # the reference's own CPU path, as child processes before anything touches the GPU
    if want_cpu:
        phase(rank, "CPU baselines (the reference on the host cores)")
    cpu_ref = cpu_baseline_reference(n=args.edge, b=args.block) if want_cpu else None
    cpu_x = cpu_baseline_configs(keys_x) if want_cpu and keys_x else {}
    # N > 1: the reference's multi-rank path (mpiexec -n N), measured by the spawning parent
    # (COSTA_BENCH_CPU_MR names its file) or, under an outside launcher, here by rank 0 -- in
    # both cases before this process touches the GPU
    cpu_mr = {}
    if rank == 0 and world > 1 and not args.no_cpu_baseline and args.workload == "pxtran":
        path = os.environ.get(CPU_MR_ENV)
        if path and os.path.exists(path):
            cpu_mr = json.load(open(path))
        else:
            phase(rank, f"CPU baselines (the reference on {world} MPI ranks)")
            cpu_mr = cpu_baseline_multirank(world, keys_x)
    import torch
    import torch.distributed as dist
    import costa_amd as costa

    costa.lib()
    if torch.cuda.device_count() < world:
        print(f"bench.py: {world} ranks but {torch.cuda.device_count()} GPU(s) visible",
              file=sys.stderr)
        raise SystemExit(2)
    device = local_rank
    torch.cuda.set_device(device)
    if world > 1:
        start_watchdog(rank, world, float(os.environ.get("COSTA_BENCH_RANK_BUDGET_S",
                                                         RUN_BUDGET_S - 30.0)))
        phase(rank, "init_process_group (gloo control plane)")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ---- communicator: RCCL unique id from rank 0, broadcast over the control plane
    if world > 1:
        uid = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            uid = torch.frombuffer(bytearray(costa.Comm.unique_id()), dtype=torch.uint8).clone()
        dist.broadcast(uid, 0)
        phase(rank, f"ncclCommInitRank (RCCL {costa.rccl_version()}, {world} ranks, device {device})")
        t0 = time.perf_counter()
        comm = costa.Comm.create(bytes(uid.numpy().tobytes()), world, rank, device)
        phase(rank, f"communicator ready: ncclCommInitRank took {(time.perf_counter() - t0) * 1e3:.1f} ms")
    else:
        comm = costa.Comm.self(device)

    # ---- workloads
    def checksum(t, mask=None):
        """order-independent checksum of a tensor's bit patterns (equal for any permutation of
        the same elements), summed over the ranks: cfg 5 'N''s bijection check, beside the
        position samples"""
        x = t.view(torch.int32 if t.element_size() == 4 else torch.int64).reshape(-1)
        if mask is not None:
            x = x[mask]
        x = x.to(torch.int64)
        v = torch.stack([x.sum(), (x * x).sum(), (x ^ (x >> 7)).sum()]).cpu()
        if world > 1:
            dist.all_reduce(v)
        return v.tolist()

    def sum_over_ranks(x: int) -> int:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.int64)
        dist.all_reduce(t)
        return int(t.item())

    gen = torch.Generator(device="cuda")
    gen.manual_seed(777 + rank)

    def bc_check(Cm, lr_c, lc_c, b, cgrid, a_of, axpby=False, al=1.0, be=0.0, kind="f64"):
        return lambda: sum_over_ranks(mismatch_bc(Cm, lr_c, lc_c, b, cgrid, a_of, gen, axpby,
                                                  al, be, kind)) == 0

    def build(kind, edge=None):
        """-> dict: layouts, tensors, op / alpha / beta, description, correctness check.
        Data: pos_values of every element's global position (seeds SEED_A / SEED_C)"""
        n, b = args.edge, args.block
        pm, pn = grid_for(world)
        pr, pc = rank // pn, rank % pn  # 'R' rank order on the pm x pn grid
        w = {"kind": kind, "check": None, "repeatable": True}
        if kind == "cfg5":
            LA, LC, A, Cm, op, al, be, wl, masks, ca = cfg5_workload(
                costa, torch, rank, world, args.cfg5_op if edge is None else edge)
            w.update(LA=LA, LC=LC, A=A, C=Cm, op=op, al=al, be=be, wl=wl, repeatable=be == 0)
            C0 = Cm.clone() if be != 0 else None
            ref = checksum(A, masks[0]) if op == "N" else None

            def check():
                good = sum_over_ranks(mismatch_arena(Cm, ca, op, gen, C0, al, be)) == 0
                if ref is not None:  # and a bit permutation of A's block elements into C's
                    good = good and checksum(Cm, masks[1]) == ref
                return good
            w["check"] = check
            return w
        if kind == "cfg3":
            # BASELINE configs[2]: pxgemr2d fp64 'N' (bit copy), 128^2 blocks, A on
            # the pm x pn grid -> C on a world x 1 grid ('R' rank order both); 32768^2 per rank
            # (65536^2 2x2 -> 4x1 at 4 ranks)
            b, e3 = 128, 32768
            M, N = e3 * pm, e3 * pn
            lr_a, lc_a = M // pm, N // pn
            lr_c, lc_c = M // world, N
            A = torch.empty(lr_a * lc_a, dtype=torch.float64, device="cuda")
            fill_bc(A, lr_a, lc_a, b, pm, pr, pn, pc, SEED_A, "f64")
            Cm = torch.zeros(lr_c * lc_c, dtype=torch.float64, device="cuda")
            LA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0,
                                           A.data_ptr(), lr_a, "C", rank)
            LC = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, world, 1, "R", 0, 0,
                                           Cm.data_ptr(), lr_c, "C", rank)
            wl = (f"pxgemr2d fp64 {M}x{N}, 128x128 blocks, {pm}x{pn} -> {world}x1 grid remap, "
                  f"op N (BASELINE configs[2])" if world > 1 else
                  f"copy slice of BASELINE configs[2]: pxgemr2d fp64 {M}x{N}, 128x128 blocks on "
                  f"one rank (1x1 -> 1x1: every tile is a local bit copy, no remap)")
            w.update(LA=LA, LC=LC, A=A, C=Cm, op="N", al=1.0, be=0.0, wl=wl, grid=f"{pm}x{pn}",
                     m=M, n=N, block=b)
            sampled = bc_check(Cm, lr_c, lc_c, b, (world, rank, 1, 0), lambda i, j: (i, j))
            w["check"] = (lambda: torch.equal(Cm, A) and sampled()) if world == 1 else sampled
            return w
        if kind == "cfg4":
            # BASELINE configs[3]: pztranu, c128, 128^2 blocks, alpha=(0.75,-0.5),
            # beta=(1.25,0.25) (C is read); `edge` = the global square edge (32768 at 8 ranks),
            # else 16384^2 per rank weak-scaled on the pm x pn grid
            b = 128
            M, N = (edge, edge) if edge else (n * pm, n * pn)
            lr_a, lc_a = M // pm, N // pn
            lr_c, lc_c = N // pm, M // pn
            A = torch.empty(lr_a * lc_a, dtype=torch.complex128, device="cuda")
            Cm = torch.empty(lr_c * lc_c, dtype=torch.complex128, device="cuda")
            fill_bc(A, lr_a, lc_a, b, pm, pr, pn, pc, SEED_A, "c128")
            fill_bc(Cm, lr_c, lc_c, b, pm, pr, pn, pc, SEED_C, "c128")
            LA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0,
                                           A.data_ptr(), lr_a, "C", rank, dtype=costa.CDOUBLE)
            LC = costa.block_cyclic_layout(N, M, b, b, 1, 1, N, M, pm, pn, "R", 0, 0,
                                           Cm.data_ptr(), lr_c, "C", rank, dtype=costa.CDOUBLE)
            al, be = complex(0.75, -0.5), complex(1.25, 0.25)
            if args.cfg4_beta0:  # A/B only: the same transpose without reading C
                be = complex(0.0, 0.0)
            wl = (f"pztranu c128 {M}x{N} on a {pm}x{pn} rank grid, 128x128 blocks, op T, "
                  f"alpha=(0.75,-0.5) beta=({be.real},{be.imag}) (BASELINE configs[3]"
                  f"{', single-GPU slice' if world == 1 else ''}"
                  f"{', weak-scaled 16384^2 per rank' if world > 1 and not edge else ''})")
            w.update(LA=LA, LC=LC, A=A, C=Cm, op="T", al=al, be=be, wl=wl, grid=f"{pm}x{pn}",
                     m=M, n=N, block=b, repeatable=False)
            # after the first call only (beta != 0: every step changes C): C = beta*C0 + alpha*A^T
            w["check"] = bc_check(Cm, lr_c, lc_c, b, (pm, pr, pn, pc), lambda i, j: (j, i),
                                  axpby=True, al=al, be=be, kind="c128")
            return w
        # pxtran: BASELINE configs[1] at one rank, weak-scaled 16384^2 per rank beyond
        M, N = n * pm, n * pn  # A: M x N on pm x pn; C = A^T: N x M on the same rank grid
        lr_a, lc_a = M // pm, N // pn
        lr_c, lc_c = N // pm, M // pn
        A = torch.empty(lr_a * lc_a, dtype=torch.float64, device="cuda")
        fill_bc(A, lr_a, lc_a, b, pm, pr, pn, pc, SEED_A, "f64")
        Cm = torch.zeros(lr_c * lc_c, dtype=torch.float64, device="cuda")
        LA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0, A.data_ptr(),
                                       lr_a, "C", rank)
        LC = costa.block_cyclic_layout(N, M, b, b, 1, 1, N, M, pm, pn, "R", 0, 0, Cm.data_ptr(),
                                       lr_c, "C", rank)
        wl = (("pxtran fp64 16384x16384, 256x256 blocks, op T, alpha=1 beta=0, "
               "1x1 grid (BASELINE configs[1])") if world == 1 else
              (f"pxtran fp64 weak-scaled: {M}x{N} on a {pm}x{pn} rank grid "
               f"(16384^2 per rank), 256x256 blocks, op T, alpha=1 beta=0"))
        w.update(LA=LA, LC=LC, A=A, C=Cm, op="T", al=1.0, be=0.0, wl=wl, grid=f"{pm}x{pn}",
                 m=M, n=N, block=b)
        sampled = bc_check(Cm, lr_c, lc_c, b, (pm, pr, pn, pc), lambda i, j: (j, i))
        w["check"] = ((lambda: torch.equal(Cm.view(n, n), A.view(n, n).t()) and sampled())
                      if world == 1 else sampled)
        return w

    def measure(w, steps, warmup, planning_modes=False):
        LA, LC, op, al, be = w["LA"], w["LC"], w["op"], w["al"], w["be"]

        def step_blocking():
            costa.transform(LA, LC, comm, op, al, be)

        def step_async():  # stream-ordered: the host queues step k+1 while step k runs
            costa.transform_async(LA, LC, comm, op, al, be)

        def timed(step, profile=True):
            costa.set_profiling(profile)
            costa.get_stats(reset=True)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            costa.synchronize(comm)
            torch.cuda.synchronize()
            barrier()
            el = max_over_ranks(time.perf_counter() - t0)
            st = costa.get_stats(reset=True)
            costa.set_profiling(False)
            return el, st

        r = {}
        # first call on these layouts: planning + descriptor upload + kernels (plan-cache miss)
        torch.cuda.synchronize()
        costa.get_stats(reset=True)
        barrier()
        t0 = time.perf_counter()
        step_blocking()
        r["first_call_ms"] = max_over_ranks(time.perf_counter() - t0) * 1e3
        st0 = costa.get_stats(reset=True)
        verified = []
        if w["check"] and not w["repeatable"]:
            verified.append(w["check"]())  # before any further call changes C
        planning = {"planner": "device" if st0["device_plans"] else "host",
                    "plan_ms": round(max_over_ranks(st0["plan_ms"]), 2)}
        if planning_modes:
            # plan-cache misses with each planner.  The first GPU plan of a process loads the
            # planner's kernels (rocPRIM sort + scan, ~15 ms with the device allocations):
            # "device_cold" is that first one, "device" the next miss on the same layouts (warm),
            # the figure DESIGN §2b tabulates
            for mode, key in ((1, "default"), (0, "host"), (2, "device_cold"), (2, "device")):
                costa.set_planner(mode)
                costa.release_caches()
                t0 = time.perf_counter()
                step_blocking()
                sm = costa.get_stats(reset=True)
                planning[key] = {"call_ms": round((time.perf_counter() - t0) * 1e3, 2),
                                 "plan_ms": round(sm["plan_ms"], 2),
                                 "planner": "device" if sm["device_plans"] else "host"}
            costa.set_planner(1)
        r["planning"] = planning
        for _ in range(warmup):
            step_blocking()
        if w["check"] and w["repeatable"]:  # correctness of what we time
            verified.append(w["check"]())
        r["el_block"], _ = timed(step_blocking, profile=False)
        for _ in range(warmup):
            step_async()
        # value: the product as shipped (phase-timing events off: recording them costs ~11 us per
        # step on cfg 2, tools/step_gap_probe.py); then the same steps again with the events on,
        # for the kernel durations (roofline.avg_launch_ms, phase_ms_per_step)
        r["el"], st_val = timed(step_async, profile=False)
        r["el_ev"], st = timed(step_async)
        assert all(st_val[k] == st[k] for k in ("local_bytes", "pack_bytes", "unpack_bytes"))
        if w["check"] and w["repeatable"]:
            verified.append(w["check"]())
        r["verified"] = all(verified) if verified else None
        if r["verified"] is False:
            raise RuntimeError(f"bench.py: wrong result for workload {w['kind']}")
        r["st"] = st
        alg_bytes = st["local_bytes"] + st["pack_bytes"] + st["unpack_bytes"]  # this rank
        total = float(alg_bytes)
        if world > 1:
            t = torch.tensor([total], dtype=torch.float64)
            dist.all_reduce(t)
            total = t.item()
        r["total_bytes"] = total
        r["value"] = total / r["el"] / 1e9
        # SURVEY §8(d) node figure: kernel time only (pack + local + unpack), summed bytes / max t
        kern_ms = (st["local_ms"] + st["pack_ms"] + st["unpack_ms"]) / steps
        r["kern_ms_max"] = max_over_ranks(kern_ms)
        r["kernel_node"] = (total / steps / (r["kern_ms_max"] * 1e-3) / 1e9
                            if r["kern_ms_max"] > 0 else None)
        # this rank's kernels against the roofline; min / max over the ranks
        own = alg_bytes / steps / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else 0.0
        r["rank_frac"] = [round(-max_over_ranks(-own) / HBM_PEAK_GBPS, 4),
                          round(max_over_ranks(own) / HBM_PEAK_GBPS, 4)]
        r["exchange_ms"] = max_over_ranks(st["exchange_ms"] / steps)
        r["kernels"] = kernels_ran(st, steps, {"pxtran": "double", "cfg3": "double", "cfg4": "cpx<double>",
                                               "cfg5": "float"}[w["kind"]])
        return r

    def summary(w, r, steps):  # one extra-config entry of the JSON line
        out = {"workload": w["wl"], "n_gpus": world, "rccl_ranks": world if world > 1 else 0,
               "steps": steps, "bytes_per_step": int(r["total_bytes"] / steps),
               "ms_per_step": round(r["el"] / steps * 1e3, 4), "GBps": round(r["value"], 2),
               "kernel_node_GBps": round(r["kernel_node"], 2) if r["kernel_node"] else None,
               "rank_kernel_frac_min_max": r["rank_frac"],
               "exchange_ms_per_step": round(r["exchange_ms"], 4),
               "phase_ms_per_step": {k: round(r["st"][k + "_ms"] / steps, 4)
                                     for k in ("pack", "local", "unpack")},
               "first_call_ms": round(r["first_call_ms"], 2), "verified": r["verified"],
               # the pass the phase (kernel) times come from, so that kernel <= step reads off
               # the entry itself
               "events_pass_ms_per_step": round(r["el_ev"] / steps * 1e3, 4),
               "kernels": r["kernels"]}
        for k in ("grid", "m", "n", "block"):
            if k in w:
                out[k] = w[k]
        return out

    phase(rank, f"build workload {args.workload}")
    wmain = build(args.workload)
    phase(rank, f"measure workload {args.workload} (first call, warmup, {args.steps} timed steps)")
    torch.cuda.synchronize()
    res = measure(wmain, args.steps, args.warmup, planning_modes=world == 1)
    el, el_block, el_ev, st = res["el"], res["el_block"], res["el_ev"], res["st"]
    total_bytes, value, kernel_node = res["total_bytes"], res["value"], res["kernel_node"]
    op, al, be, wl = wmain["op"], wmain["al"], wmain["be"], wmain["wl"]
    A, Cm = wmain["A"], wmain["C"]
    n, b = args.edge, args.block
    pm, pn = grid_for(world)
    M, N = wmain.get("m", 0), wmain.get("n", 0)

    if rank == 0:  # what the watchdog reports should a later phase hang
        _partial_line.update({
            "value": round(value, 2), "pct_hbm_peak": round(100 * value / (HBM_PEAK_GBPS * world), 2),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "strong" if args.workload == "cfg5" else "weak", "vs_baseline": None,
            "dtype": {"pxtran": "f64", "cfg3": "f64", "cfg4": "c128", "cfg5": "f32"}[args.workload],
            "config": {"workload": wmain["wl"]}, "verified": res["verified"],
            "partial": "the headline was measured; a later phase did not finish"})

    # dominant kernel: the launch list moving the most bytes on this rank
    kern = max([("local", st["local_bytes"], st["local_ms"], st["local_launches"]),
                ("pack", st["pack_bytes"], st["pack_ms"], st["pack_launches"]),
                ("unpack", st["unpack_bytes"], st["unpack_ms"], st["unpack_launches"])],
               key=lambda x: x[1])
    name, kbytes, kms, kl = kern
    per_launch = kbytes / max(kl, 1)
    avg_ms = kms / max(kl, 1)
    achieved = per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic, traffic_src = measured_traffic(int(per_launch))
    kdt = {"pxtran": "double", "cfg3": "double", "cfg4": "cpx<double>", "cfg5": "float"}[args.workload]
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": (f"tile_kernel<{kdt}> ({name} list)" if args.workload != "cfg5" else
                       f"cblock_kernel<float> + tiny_kernel<float> ({name} list: destination-block "
                       f"groups, the few ops outside them as wavefront pieces)"),
            "bytes_per_launch": int(per_launch),
            "avg_launch_ms": round(avg_ms, 4),
            "kernels": res["kernels"]}

    roof.update(pass_fracs(per_launch, kl / args.steps, avg_ms, el / args.steps * 1e3,
                           el_ev / args.steps * 1e3))
    # the copy ceiling of the same bytes on this box, measured after the timed
    # region (it overwrites C, whose checks have run)
    if world == 1 and args.workload == "pxtran":
        torch.cuda.synchronize()
        cc = copy_ceiling(A, Cm, col_bytes=(M // pm) * 8)
        best = max((v.get("GBps", 0.0) for v in cc.values()), default=0.0)
        cc["best_GBps"] = best
        cc["note"] = ("plain copies of the headline's A into C (2 GiB read + 2 GiB written), "
                      "median of 20 event-timed repetitions each, measured in this process "
                      "after the timed region")
        roof["copy_ceiling"] = cc
        roof["frac_of_ceiling"] = round(achieved / best, 4) if best > 0 else None

    # end-to-end from host memory (H2D + kernels [+ RCCL] + D2H), reported, never `value`: each
    # rank's local A and C in host memory, the same algorithmic bytes as the device legs
    e2e = None
    if not args.no_e2e and args.workload == "pxtran":
        import numpy as np
        phase(rank, "end-to-end from host memory")
        bytes_call = total_bytes / args.steps  # all ranks
        ha = A.cpu().numpy()
        hc = np.zeros(Cm.numel())
        HA, HC = host_layouts(costa, ha, hc, M, N, b, pm, pn, rank)

        def leg(LA, LC, hcx, hax):
            def start_stats():
                costa.set_profiling(True)
                costa.get_stats(reset=True)
            gb, ms, ok = e2e_leg(lambda: costa.transform(LA, LC, comm, "T", 1.0, 0.0), hcx,
                                 lambda: host_c_check(hcx, hax, M, N, b, pm, pn, rank, world, gen,
                                                      sum_over_ranks),
                                 bytes_call, barrier, max_over_ranks, before_timed=start_stats)
            sx = costa.get_stats(reset=True)
            costa.set_profiling(False)
            calls = max(1, sx["transforms"])  # the timed calls
            return gb, ms, ok, sx, calls

        res_e = {}
        for mode in ((1, 0) if world == 1 else (1,)):  # pipelined (default), then the mirror
            costa.set_host_staging(mode)
            gb, ms, ok, sx, calls = leg(HA, HC, hc, ha)
            res_e[mode] = {"GBps_algorithmic": gb, "ms_per_call": ms,
                           "h2d_ms": round(sx["h2d_ms"] / calls, 2),
                           "d2h_ms": round(sx["d2h_ms"] / calls, 2),
                           "kernel_ms": round((sx["local_ms"] + sx["unpack_ms"]) / calls, 3)}
            if mode == 1:
                res_e[mode].update({"groups": sx["host_groups"] // calls, "verified": ok})
                if world > 1:
                    res_e[mode]["exchange_ms"] = round(sx["exchange_ms"] / calls, 2)
            if ok is False:
                raise RuntimeError("bench.py: wrong end-to-end result (host staging mode %d)" % mode)
        costa.set_host_staging(1)
        # the same from page-locked host arrays (hipHostMalloc via torch's pinned allocator):
        # groups whose footprints are rectangles of the caller's arrays move by strided DMA
        # between those arrays and HBM (pack / unpack groups included), no host copies
        tpa = torch.empty(ha.nbytes, dtype=torch.uint8, pin_memory=True)
        tpc = torch.empty(hc.nbytes, dtype=torch.uint8, pin_memory=True)
        pa, pc = tpa.numpy().view(ha.dtype), tpc.numpy().view(hc.dtype)
        pa[:] = ha
        PA, PC = host_layouts(costa, pa, pc, M, N, b, pm, pn, rank)
        gb, ms, okp, sx, calls = leg(PA, PC, pc, pa)
        pinned = {"GBps_algorithmic": gb, "ms_per_call": ms,
                  "h2d_ms": round(sx["h2d_ms"] / calls, 2), "d2h_ms": round(sx["d2h_ms"] / calls, 2),
                  "direct_dma": sx["host_direct"] == calls,
                  "direct_groups": f"{sx['host_direct_groups'] // calls} of {sx['host_groups'] // calls}",
                  "verified": okp}
        if world > 1:
            pinned["exchange_ms"] = round(sx["exchange_ms"] / calls, 2)
        if okp is False:
            raise RuntimeError("bench.py: wrong end-to-end result (page-locked host memory)")
        del PA, PC, tpa, tpc, pa, pc
        e2e = dict(res_e[1])
        e2e["pinned_host"] = pinned
        if world == 1:
            e2e["mirror"] = res_e[0]
        e2e["note"] = ("each rank's local A and C in pageable host memory (numpy), "
                       f"{2 * ha.nbytes / 2**30:.0f} GiB a rank over PCIe; the algorithmic bytes of "
                       "the device legs over the max time of a blocking call over the ranks. "
                       "Pipelined (default): 64 MiB tile groups, host gather -> H2D -> tile kernels "
                       "-> D2H -> host scatter, both copy directions at once (h2d_ms / d2h_ms = span "
                       "of each copy stream)"
                       + (", pack groups gathered straight into the send buffer, RCCL exchange in "
                          "rounds, unpack groups scattered back" if world > 1 else "")
                       + ". pinned_host: the same matrices in page-locked host memory, groups moved "
                         "by strided DMA straight between the caller's arrays and HBM where their "
                         "footprints are rectangles (direct_groups)"
                       + (". mirror: H2D of A's range, kernel, D2H of C's range (C not uploaded: "
                          "beta=0 and every byte of it is overwritten)" if world == 1 else ""))
        del ha, hc, HA, HC

    # fixed cost of one blocking transform call (plan-cache hit, one 16x16 tile)
    overhead_us = None
    if world == 1:
        # (16 x 16: a wavefront-path op, so that the profiler's per-kernel averages of the
        # tile_kernel stay those of the workload's launches)
        ta = torch.zeros(16 * 16, dtype=torch.float64, device="cuda")
        tc = torch.zeros(16 * 16, dtype=torch.float64, device="cuda")
        SA = costa.block_cyclic_layout(16, 16, 16, 16, 1, 1, 16, 16, 1, 1, "R", 0, 0,
                                       ta.data_ptr(), 16, "C", 0)
        SC = costa.block_cyclic_layout(16, 16, 16, 16, 1, 1, 16, 16, 1, 1, "R", 0, 0,
                                       tc.data_ptr(), 16, "C", 0)
        for _ in range(10):
            costa.transform(SA, SC, comm, "T", 1.0, 0.0)
        t1 = time.perf_counter()
        for _ in range(200):
            costa.transform(SA, SC, comm, "T", 1.0, 0.0)
        overhead_us = round((time.perf_counter() - t1) / 200 * 1e6, 1)

    # BASELINE's other configurations (plan_x above; the driver runs only `bench.py --gpus N`)
    extra = {}
    if keys_x:
        for key in ("LA", "LC", "check"):
            wmain.pop(key, None)
        for key, kind, edge in keys_x:
            costa.release_caches()
            torch.cuda.empty_cache()
            phase(rank, f"extra config {kind}:{edge}: build")
            wx = build(kind, edge)
            phase(rank, f"extra config {kind}:{edge}: measure")
            ksteps = max(1, min(args.steps, 5 if kind != "cfg5" else 10))
            rx = measure(wx, ksteps, 1)
            extra[key] = summary(wx, rx, ksteps)
            if key in cpu_x:
                extra[key]["cpu_baseline"] = cpu_x[key]
            elif key in cpu_mr:
                extra[key]["cpu_baseline"] = cpu_mr[key]
            del wx, rx
            costa.release_caches()
            torch.cuda.empty_cache()
            if rank == 0:
                _partial_line.setdefault("baseline_configs", {})[key] = extra[key]

    phase(rank, "report")
    cpu = None
    if want_cpu:
        port = cpu_baseline(n=n, b=b)  # our restatement of the tile loop (oracle/), same tiles
        cpu = cpu_ref or port
        if cpu_ref:
            cpu["port"] = {k: port[k] for k in ("value", "cores", "kind", "sample")}
        else:
            cpu["note"] = "REFERENCE BINARY ABSENT: this is our restatement (kind 'port')"
    elif cpu_mr.get("headline"):
        cpu = cpu_mr["headline"]

    if rank == 0:
        def js(x):  # complex scalars as [re, im]
            return [x.real, x.imag] if isinstance(x, complex) else x
        cfg = {"workload": wl, "op": op, "alpha": js(al), "beta": js(be),
               "parallelism": f"{world} rank(s), one per GPU, RCCL send/recv exchange",
               "bytes_per_step": int(total_bytes / args.steps)}
        if args.workload in ("pxtran", "cfg3", "cfg4"):
            cfg.update({"m": M, "n": N, "block": wmain.get("block", b), "grid": f"{pm}x{pn}"})
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "pct_hbm_peak": round(100 * value / (HBM_PEAK_GBPS * world), 2),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "cfg5" else "weak",
            "vs_baseline": None,
            "dtype": {"pxtran": "f64", "cfg3": "f64", "cfg4": "c128", "cfg5": "f32"}[args.workload],
            "data": ("synthetic, device-resident: every element a hash of its global (row, col), "
                     "uniform on +-[1, 2); checks sample positions bit for bit"),
            "config": cfg,
            "roofline": roof,
            "cpu_baseline": cpu,
            "e2e_host": e2e,
            "verified": res["verified"],
            "call_overhead_us": overhead_us,
            "first_call_ms": round(res["first_call_ms"], 2),  # plan-cache miss
            "planning": res["planning"],
            "blocking": {"ms_per_step": round(el_block / args.steps * 1e3, 4),
                         "GBps": round(total_bytes / el_block / 1e9, 2),
                         "note": "costa_hip_transform (reference semantics: host waits for C)"},
            "value_mode": ("costa_hip_transform_async steps, stream-ordered, one sync at the end; "
                           "phase-timing events off (the shipped default)"),
            "with_phase_events": {"ms_per_step": round(el_ev / args.steps * 1e3, 4),
                                  "GBps": round(total_bytes / el_ev / 1e9, 2),
                                  "note": "second pass of the same K steps with a HIP event "
                                          "pair around every phase: the source of the kernel "
                                          "durations (roofline.avg_launch_ms)"},
            "kernel_node_GBps": round(kernel_node, 2) if kernel_node else None,
            "rank_kernel_frac_min_max": res["rank_frac"],
            "phase_ms_per_step": {k: round(st[k + "_ms"] / args.steps, 4)
                                  for k in ("pack", "local", "unpack", "exchange")},
        }
        if extra:
            line["baseline_configs"] = extra
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
