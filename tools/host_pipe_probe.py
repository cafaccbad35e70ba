#!/usr/bin/env python3
"""Host-resident end-to-end probe: cfg 2 geometry (16384^2 fp64 'T', 256^2 blocks) from pageable
numpy arrays, pipelined staging under several slot sizes / host thread counts, plus the mirror
scheme.  One child process per setting (the knobs are read once per process).
    python3 tools/host_pipe_probe.py            (parent)
    python3 tools/host_pipe_probe.py child      (one measurement, knobs from the env)
    python3 tools/host_pipe_probe.py nt         (slot sizes x COSTA_HOST_NT: streaming or cached
                                                 stores of the gather / scatter, two passes)"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child():
    import numpy as np
    import costa_amd as costa
    n, b = int(os.environ.get("PROBE_N", "16384")), 256
    mode = int(os.environ.get("PROBE_MODE", "1"))
    costa.lib()
    costa.set_host_staging(mode)
    ha = np.random.default_rng(1).standard_normal(n * n)
    hc = np.zeros(n * n)
    A = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, ha, n, "C", 0)
    C = costa.block_cyclic_layout(n, n, b, b, 1, 1, n, n, 1, 1, "R", 0, 0, hc, n, "C", 0)
    comm = costa.Comm.self(0)
    costa.transform(A, C, comm, "T", 1.0, 0.0)
    ok = bool(np.array_equal(hc.reshape(n, n), ha.reshape(n, n).T))
    costa.transform(A, C, comm, "T", 1.0, 0.0)
    ts = []
    for _ in range(4):
        t0 = time.perf_counter()
        costa.transform(A, C, comm, "T", 1.0, 0.0)
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    print(json.dumps({"mode": mode, "loopback": os.environ.get("COSTA_LOOPBACK", "0"),
                      "slot_mib": os.environ.get("COSTA_HOST_SLOT_MIB", "64"),
                      "threads": os.environ.get("COSTA_HOST_THREADS", "16"),
                      "nt": os.environ.get("COSTA_HOST_NT", "3"),
                      "ms_best": round(t * 1e3, 2), "ms_all": [round(x * 1e3, 2) for x in ts],
                      "GBps_alg": round(2 * ha.nbytes / t / 1e9, 2), "verified": ok}), flush=True)


def main(sweep=None):
    settings = [{"PROBE_MODE": "0"}]
    for slot, th in (("32", "16"), ("64", "16"), ("128", "16")):
        settings.append({"PROBE_MODE": "1", "COSTA_HOST_SLOT_MIB": slot, "COSTA_HOST_THREADS": th})
    # the exchange path on one GPU: every tile packed, sent to itself over RCCL and unpacked
    for mode in ("0", "1"):
        settings.append({"PROBE_MODE": mode, "COSTA_LOOPBACK": "1"})
    if sweep == "nt":
        settings = [{"PROBE_MODE": "1", "COSTA_HOST_SLOT_MIB": slot, "COSTA_HOST_NT": nt}
                    for _ in range(2) for slot in ("16", "32", "64") for nt in ("3", "2", "1", "0")]
    for s in settings:
        env = dict(os.environ, COSTA_HOST_PIPE_TRACE="1", COSTA_TUNING="1", **s)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env,
                           capture_output=True, text=True, timeout=240)
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        traces = [l for l in r.stderr.splitlines() if "host pipe" in l]
        print(lines[-1] if lines else f"FAILED {s} rc={r.returncode} {r.stderr[-400:]}", flush=True)
        if traces:
            print("   ", traces[-1], flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child()
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else None)
