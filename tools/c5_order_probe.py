#!/usr/bin/env python3
"""Probe (not product): cfg 5 wavefront kernel time against the op order (the planner's
locality hint).  Environment knobs are read once per process, so run one process per setting:
    COSTA_ORDER_BAND=<rows> COSTA_TINY_XCD=0|1 python tools/c5_order_probe.py N|T
Host planner, 20 timed launches after 3 warm-ups; prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import costa_amd as costa  # noqa: E402
from bench import cfg5_workload  # noqa: E402

op_name = sys.argv[1] if len(sys.argv) > 1 else "T"
costa.lib()
torch.cuda.set_device(0)
costa.set_planner(int(os.environ.get("PROBE_PLANNER", "0")))
LA, LC, A, C, op, al, be, _ = cfg5_workload(costa, torch, 0, 1, op_name)
comm = costa.Comm.self(0)
for _ in range(3):
    costa.transform_async(LA, LC, comm, op, al, be)
costa.synchronize(comm)
costa.set_profiling(True)
costa.get_stats(reset=True)
steps = 20
for _ in range(steps):
    costa.transform_async(LA, LC, comm, op, al, be)
costa.synchronize(comm)
st = costa.get_stats(reset=True)
ms = st["local_ms"] / steps
print(json.dumps({"op": op_name, "band": os.environ.get("COSTA_ORDER_BAND", "0"),
                  "xcd": os.environ.get("COSTA_TINY_XCD", "0"), "kernel_ms": round(ms, 4),
                  "GBps": round(st["local_bytes"] / steps / (ms * 1e-3) / 1e9, 1)}), flush=True)
