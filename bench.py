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
Timing: W untimed steps; then barrier + device sync, K steps, device sync + barrier; max over
ranks.  value = algorithmic bytes of all ranks / that time (read + write of every
element moved, + read of C when beta != 0).  Rank 0 prints ONE JSON line.

roofline: the dominant kernel's algorithmic bytes per launch / its average duration from
HIP events recorded on the stream it runs on (costa_hip_get_stats), against 8 TB/s.  Those
events are recorded in a second pass of the same K steps: in the `value` pass they are off, as
they are in the shipped library (each event pair adds ~11 us to a 0.83 ms cfg 2 step).
cpu_baseline: the oracle's restatement of the reference's OpenMP tile loop (256x256-blocked
transpose, OpenMP over tiles) on a bounded sample of the same tiles, rank 0 at N = 1.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def grid_for(n: int):
    pm = int(math.isqrt(n))
    while n % pm:
        pm -= 1
    return pm, n // pm


def measured_traffic(alg_bytes: int):
    """HBM bytes per launch phase of this workload, from the newest committed rocprofv3 PMC
    pass of this same bench command (profiles/<tag>/pmc_*.json, one per workload, written by
    tools/save_profiles.py with the gfx950 FETCH_SIZE correction; matched on the algorithmic
    bytes per launch).  PMC counters cannot be read from inside this process, so they come
    from that separate pass."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_*.json"))):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("bytes_per_launch_alg") == alg_bytes and d.get("hbm_bytes_per_launch_corrected"):
            best = (d["hbm_bytes_per_launch_corrected"], os.path.relpath(p, ROOT))
    return best if best else (None, None)


def cpu_baseline(n=16384, b=256, slab_cols=2048, target_s=10.0):
    """Oracle restatement of the reference tile loop on a 16384 x 2048 column slab of A
    (512 tiles of 256^2 fp64, 256 MiB in / 256 MiB out), repeated for ~target_s seconds."""
    import numpy as np
    import oracle
    threads = min(16, os.cpu_count() or 1)
    a = np.random.default_rng(1).standard_normal(n * slab_cols)  # col-major, ld n
    c = np.zeros(slab_cols * n)                                  # col-major, ld slab_cols
    tiles = []
    for j in range(slab_cols // b):
        for i in range(n // b):
            # A tile (i, j) -> C tile (j, i): (src_off, lds, dst_off, ldd, F, S)
            tiles.append((i * b + j * b * n, n, j * b + i * b * slab_cols, slab_cols, b, b))
    tiles = np.array(tiles, np.int64)
    oracle.transform_tiles(1, 1, 0, 1.0, 0.0, a, c, tiles, threads)  # warm-up, first touch
    reps, t0 = 0, time.perf_counter()
    while True:
        oracle.transform_tiles(1, 1, 0, 1.0, 0.0, a, c, tiles, threads)
        reps += 1
        el = time.perf_counter() - t0
        if el >= target_s or reps >= 1000:
            break
    ok = np.array_equal(c.reshape(n, slab_cols).T, a.reshape(slab_cols, n))
    bytes_per = 2 * a.nbytes
    return {"value": round(bytes_per * reps / el / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "sample": f"{len(tiles)} tiles of 256x256 fp64 ('T', alpha=1, beta=0; a 16384x2048 "
                      f"slab of cfg 2), {reps} passes in {el:.1f} s, oracle/costa_oracle.c "
                      f"oracle_transform_tiles, OpenMP {threads} threads, verified={ok}"}


def cpu_baseline_reference(n=16384, b=256, slab_cols=2048, target_s=10.0):
    """The REFERENCE itself on the host cores: oracle/_ref/ref_harness (eth-cscs/COSTA compiled
    from its own sources by oracle/Makefile; the binary travels with the repo snapshot) runs
    costa::transform 'T' (alpha 1, beta 0) on a 16384 x 2048 fp64 slab in 256^2 blocks (the
    same 512 tiles as cpu_baseline) for ~target_s seconds.  Started as a child process before
    this process touches the GPU.  None when the binary is absent."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        return None
    threads = min(16, os.cpu_count() or 1)
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    try:
        r = subprocess.run([exe, "bench", str(n), str(slab_cols), str(b), str(target_s)],
                           capture_output=True, text=True, timeout=6 * target_s + 120, env=env)
        d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    except Exception:
        return None
    if r.returncode != 0 or not d.get("verified"):
        return None
    return {"value": round(d["GBps"], 3), "unit": "GB/s", "cores": d["threads"], "kind": "reference",
            "sample": f"{n}x{slab_cols} fp64 slab, {b}x{b} blocks on one rank: the reference's "
                      f"costa::transform 'T' (alpha=1, beta=0; planning included, as every "
                      f"reference call re-plans), {d['reps']} calls in {d['seconds']:.1f} s, "
                      f"OpenMP {d['threads']} threads, verified C == A^T"}


def cfg5_workload(costa, torch, rank, world, op):
    """BASELINE configs[4]: fp32 16384^2 custom_layout; A tile edges uniform in
    [8, 96] (seeds 0xC5A1 rows / 0xC5A2 cols), C edges uniform in [16, 160] (0xC5A3 / 0xC5A4),
    owners uniform over the ranks (0xC5A5 for A, 0xC5A6 for C); every owned block is its own
    column-major buffer (ld = rows) in a 256-byte-aligned arena.  numpy PCG64 streams are used
    for the draws.  op 'N' alpha=1 beta=0, or the 'T' variant alpha=-0.5 beta=2."""
    import numpy as np
    n = 16384

    def splits(seed, lo, hi):
        r = np.random.default_rng(seed)
        s = [0]
        while s[-1] < n:
            s.append(min(n, s[-1] + int(r.integers(lo, hi + 1))))
        return s

    ars, acs = splits(0xC5A1, 8, 96), splits(0xC5A2, 8, 96)
    crs, ccs = splits(0xC5A3, 16, 160), splits(0xC5A4, 16, 160)
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
    g = torch.Generator(device="cuda")
    g.manual_seed(99 + rank)
    A = torch.rand(an, dtype=torch.float32, device="cuda", generator=g)
    C = torch.rand(cn, dtype=torch.float32, device="cuda", generator=g)
    pa, pc = A.data_ptr(), C.data_ptr()
    LA = costa.custom_layout(len(ars) - 1, len(acs) - 1, ars, acs, aown,
                             [(pa + 4 * o, r, i, j) for o, r, i, j in ab], "C", costa.FLOAT)
    LC = costa.custom_layout(len(crs) - 1, len(ccs) - 1, crs, ccs, cown,
                             [(pc + 4 * o, r, i, j) for o, r, i, j in cb], "C", costa.FLOAT)
    al, be = (1.0, 0.0) if op == "N" else (-0.5, 2.0)
    wl = (f"costa::custom_layout fp32 16384x16384, irregular tiles (A edges 8-96: "
          f"{len(ars) - 1}x{len(acs) - 1} blocks, C edges 16-160: {len(crs) - 1}x{len(ccs) - 1}), "
          f"owners uniform over {world} rank(s), op {op} (BASELINE configs[4])")
    return LA, LC, A, C, op, al, be, wl


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
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    want_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "pxtran"
    # the reference's own CPU path, as a child process before anything touches the GPU
    cpu_ref = cpu_baseline_reference(n=args.edge, b=args.block) if want_cpu else None
    import torch
    import torch.distributed as dist
    import costa_amd as costa

    costa.lib()
    device = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    if world > 1:
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
        comm = costa.Comm.create(bytes(uid.numpy().tobytes()), world, rank, device)
    else:
        comm = costa.Comm.self(device)

    # ---- workload
    n, b = args.edge, args.block
    pm, pn = grid_for(world)
    M, N = n * pm, n * pn  # A: M x N on pm x pn; C = A^T: N x M on the same rank grid
    if args.workload == "cfg5":
        LA, LC, A, Cm, op, al, be, wl = cfg5_workload(costa, torch, rank, world, args.cfg5_op)
        check = None
    elif args.workload == "cfg3":
        # BASELINE configs[2]: pxgemr2d fp64 'N' (bit copy), 128^2 blocks, A on
        # the pm x pn grid -> C on a world x 1 grid ('R' rank order both); 32768^2 per rank
        b, e3 = 128, 32768
        M, N = e3 * pm, e3 * pn
        lr_a, lc_a = M // pm, N // pn
        lr_c, lc_c = M // world, N
        g = torch.Generator(device="cuda")
        g.manual_seed(3333 + rank)
        A = torch.rand(lr_a * lc_a, dtype=torch.float64, device="cuda", generator=g)
        Cm = torch.zeros(lr_c * lc_c, dtype=torch.float64, device="cuda")
        LA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0, A.data_ptr(),
                                       lr_a, "C", rank)
        LC = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, world, 1, "R", 0, 0, Cm.data_ptr(),
                                       lr_c, "C", rank)
        op, al, be = "N", 1.0, 0.0
        wl = (f"pxgemr2d fp64 {M}x{N}, 128x128 blocks, {pm}x{pn} -> {world}x1 grid remap, op N "
              f"(BASELINE configs[2]{', single-GPU slice' if world == 1 else ''})")

        def check():
            assert torch.equal(Cm, A), "pxgemr2d copy wrong"
    elif args.workload == "cfg4":
        # BASELINE configs[3]: pztranu, c128, 128^2 blocks, alpha=(0.75,-0.5),
        # beta=(1.25,0.25) (C is read); per rank 16384^2, weak-scaled on the pm x pn grid
        b = 128
        lr_a, lc_a = M // pm, N // pn
        lr_c, lc_c = N // pm, M // pn
        g = torch.Generator(device="cuda")
        g.manual_seed(4321 + rank)
        A = torch.rand(lr_a * lc_a, dtype=torch.complex128, device="cuda", generator=g)
        Cm = torch.rand(lr_c * lc_c, dtype=torch.complex128, device="cuda", generator=g)
        LA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0, A.data_ptr(),
                                       lr_a, "C", rank, dtype=costa.CDOUBLE)
        LC = costa.block_cyclic_layout(N, M, b, b, 1, 1, N, M, pm, pn, "R", 0, 0, Cm.data_ptr(),
                                       lr_c, "C", rank, dtype=costa.CDOUBLE)
        op, al, be = "T", complex(0.75, -0.5), complex(1.25, 0.25)
        wl = (f"pztranu c128 {M}x{N} on a {pm}x{pn} rank grid (16384^2 per rank), 128x128 "
              f"blocks, op T, alpha=(0.75,-0.5) beta=(1.25,0.25) (BASELINE configs[3], "
              f"{'single-GPU slice' if world == 1 else 'weak-scaled'})")
        C0 = Cm.clone() if world == 1 else None

        def check():  # after the first call only (beta != 0: every step changes C)
            k = torch.randint(0, n * n, (100000,), device="cuda")
            i, j = k % n, k // n  # C(i, j) at i + j*n; A(j, i) at j + i*n
            exp = be * C0[k] + al * A[j + i * n]
            assert torch.allclose(Cm[k], exp, rtol=1e-13, atol=1e-13), "cfg4 result wrong"
    else:
        lr_a, lc_a = M // pm, N // pn
        lr_c, lc_c = N // pm, M // pn
        g = torch.Generator(device="cuda")
        g.manual_seed(1234 + rank)
        A = torch.rand(lr_a * lc_a, dtype=torch.float64, device="cuda", generator=g)
        Cm = torch.zeros(lr_c * lc_c, dtype=torch.float64, device="cuda")
        LA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0, A.data_ptr(),
                                       lr_a, "C", rank)
        LC = costa.block_cyclic_layout(N, M, b, b, 1, 1, N, M, pm, pn, "R", 0, 0, Cm.data_ptr(),
                                       lr_c, "C", rank)
        op, al, be = "T", 1.0, 0.0
        wl = (("pxtran fp64 16384x16384, 256x256 blocks, op T, alpha=1 beta=0, "
               "1x1 grid (BASELINE configs[1])") if world == 1 else
              (f"pxtran fp64 weak-scaled: {M}x{N} on a {pm}x{pn} rank grid "
               f"(16384^2 per rank), 256x256 blocks, op T, alpha=1 beta=0"))

        def check():
            assert torch.equal(Cm.view(n, n), A.view(n, n).t()), "transpose result wrong"
    torch.cuda.synchronize()

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
        for _ in range(args.steps):
            step()
        costa.synchronize(comm)
        torch.cuda.synchronize()
        barrier()
        el = max_over_ranks(time.perf_counter() - t0)
        st = costa.get_stats(reset=True)
        costa.set_profiling(False)
        return el, st

    # first call on these layouts: planning + descriptor upload + kernels (plan-cache miss)
    costa.get_stats(reset=True)
    barrier()
    t0 = time.perf_counter()
    step_blocking()
    first_call_ms = max_over_ranks(time.perf_counter() - t0) * 1e3
    st0 = costa.get_stats(reset=True)
    repeatable = args.workload != "cfg4"  # beta != 0: only the first call's result is known
    if world == 1 and check and not repeatable:
        check()  # before any further call changes C
    planning = {"planner": "device" if st0["device_plans"] else "host",
                "plan_ms": round(st0["plan_ms"], 2)}
    if world == 1:  # warm plan-cache misses with each planner (the first call pays one-time costs)
        for mode, key in ((1, "default"), (0, "host"), (2, "device")):
            costa.set_planner(mode)
            costa.release_caches()
            t0 = time.perf_counter()
            step_blocking()
            sm = costa.get_stats(reset=True)
            planning[key] = {"call_ms": round((time.perf_counter() - t0) * 1e3, 2),
                             "plan_ms": round(sm["plan_ms"], 2),
                             "planner": "device" if sm["device_plans"] else "host"}
        costa.set_planner(1)
    for _ in range(args.warmup):
        step_blocking()
    if world == 1 and check and repeatable:  # correctness of what we time
        check()
    el_block, _ = timed(step_blocking, profile=False)
    for _ in range(args.warmup):
        step_async()
    # value: the product as shipped (phase-timing events off: recording them costs ~11 us per
    # step on cfg 2, tools/step_gap_probe.py); then the same K steps again with the events on,
    # for the kernel durations (roofline.avg_launch_ms, phase_ms_per_step)
    el, st_val = timed(step_async, profile=False)
    el_ev, st = timed(step_async)
    assert all(st_val[k] == st[k] for k in ("local_bytes", "pack_bytes", "unpack_bytes"))
    if world == 1 and check and repeatable:
        check()

    alg_bytes = st["local_bytes"] + st["pack_bytes"] + st["unpack_bytes"]  # this rank, K steps
    total_bytes = alg_bytes
    if world > 1:
        t = torch.tensor([float(alg_bytes)], dtype=torch.float64)
        dist.all_reduce(t)
        total_bytes = t.item()
    value = total_bytes / el / 1e9
    # SURVEY §8(d) node figure: kernel time only (pack + local + unpack), summed bytes / max t
    kern_ms = (st["local_ms"] + st["pack_ms"] + st["unpack_ms"]) / args.steps
    kern_ms = max_over_ranks(kern_ms)
    kernel_node = total_bytes / args.steps / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else None

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
                       f"tiny_kernel<float> ({name} list: every op is below the large shape)"),
            "bytes_per_launch": int(per_launch),
            "avg_launch_ms": round(avg_ms, 4)}

    # end-to-end from host memory (H2D + kernels + D2H), reported, never `value`
    e2e = None
    if not args.no_e2e and world == 1 and args.workload == "pxtran":
        import numpy as np
        ha = A.cpu().numpy()
        hc = np.zeros_like(ha)
        HA = costa.block_cyclic_layout(M, N, b, b, 1, 1, M, N, pm, pn, "R", 0, 0, ha, M, "C", rank)
        HC = costa.block_cyclic_layout(N, M, b, b, 1, 1, N, M, pm, pn, "R", 0, 0, hc, N, "C", rank)
        res = {}
        for mode in (1, 0):  # pipelined host staging (default), then the mirror scheme
            costa.set_host_staging(mode)
            hc[:] = 0
            costa.transform(HA, HC, comm, "T", 1.0, 0.0)  # plan + staging allocation
            ok = bool(np.array_equal(hc.reshape(N, M), ha.reshape(N, M).T)) if mode == 1 else None
            costa.set_profiling(True)
            costa.get_stats(reset=True)
            reps, t1 = 3, time.perf_counter()
            for _ in range(reps):
                costa.transform(HA, HC, comm, "T", 1.0, 0.0)
            te = (time.perf_counter() - t1) / reps
            sx = costa.get_stats(reset=True)
            costa.set_profiling(False)
            res[mode] = {"GBps_algorithmic": round(2 * ha.nbytes / te / 1e9, 2),
                         "ms_per_call": round(te * 1e3, 2),
                         "h2d_ms": round(sx["h2d_ms"] / reps, 2),
                         "d2h_ms": round(sx["d2h_ms"] / reps, 2),
                         "kernel_ms": round(sx["local_ms"] / reps, 3)}
            if mode == 1:
                res[mode].update({"groups": sx["host_groups"] // reps, "verified": ok})
        costa.set_host_staging(1)
        e2e = dict(res[1])
        e2e["mirror"] = res[0]
        e2e["note"] = ("pageable host A and C (numpy), 2 x 2 GiB over PCIe. Pipelined (default): "
                       "64 MiB tile groups, host gather -> H2D -> tile kernels -> D2H -> host "
                       "scatter, both copy directions at once (h2d_ms/d2h_ms = span of each "
                       "copy stream). mirror: H2D of A's range, kernel, D2H of C's range "
                       "(C not uploaded: beta=0 and every byte of it is overwritten)")

    # fixed cost of one blocking transform call (plan-cache hit, one 64x64 tile)
    overhead_us = None
    if world == 1:
        ta = torch.zeros(64 * 64, dtype=torch.float64, device="cuda")
        tc = torch.zeros(64 * 64, dtype=torch.float64, device="cuda")
        SA = costa.block_cyclic_layout(64, 64, 64, 64, 1, 1, 64, 64, 1, 1, "R", 0, 0,
                                       ta.data_ptr(), 64, "C", 0)
        SC = costa.block_cyclic_layout(64, 64, 64, 64, 1, 1, 64, 64, 1, 1, "R", 0, 0,
                                       tc.data_ptr(), 64, "C", 0)
        for _ in range(10):
            costa.transform(SA, SC, comm, "T", 1.0, 0.0)
        t1 = time.perf_counter()
        for _ in range(200):
            costa.transform(SA, SC, comm, "T", 1.0, 0.0)
        overhead_us = round((time.perf_counter() - t1) / 200 * 1e6, 1)

    cpu = None
    if want_cpu:
        port = cpu_baseline(n=n, b=b)  # our restatement of the tile loop (oracle/), same tiles
        cpu = cpu_ref or port
        if cpu_ref:
            cpu["port"] = {k: port[k] for k in ("value", "cores", "kind", "sample")}

    if rank == 0:
        def js(x):  # complex scalars as [re, im]
            return [x.real, x.imag] if isinstance(x, complex) else x
        cfg = {"workload": wl, "op": op, "alpha": js(al), "beta": js(be),
               "parallelism": f"{world} rank(s), one per GPU, RCCL send/recv exchange",
               "bytes_per_step": int(total_bytes / args.steps)}
        if args.workload in ("pxtran", "cfg3", "cfg4"):
            cfg.update({"m": M, "n": N, "block": b, "grid": f"{pm}x{pn}"})
        line = {
            "metric": "GB/s device-resident tile pack+transpose+unpack (fp64), % HBM peak",
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
            "data": "synthetic (uniform random, device-resident)",
            "config": cfg,
            "roofline": roof,
            "cpu_baseline": cpu,
            "e2e_host": e2e,
            "call_overhead_us": overhead_us,
            "first_call_ms": round(first_call_ms, 2),  # plan-cache miss: planning + upload + kernels
            "planning": planning,
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
            "phase_ms_per_step": {k: round(st[k + "_ms"] / args.steps, 4)
                                  for k in ("pack", "local", "unpack", "exchange")},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
