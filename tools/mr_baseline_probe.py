"""Probe (not product): the reference's multi-rank CPU baselines bench.py puts beside an N-rank
line (bench.cpu_baseline_multirank: oracle/_ref/ref_harness bench_mr under mpiexec -n N), run on
the GPU box's host without touching the GPU -- does MPICH start there, how long does each take,
what rates come out.  The 8-GPU node is the driver's; this rehearses the same child processes.
    python tools/mr_baseline_probe.py [N ...]   (default 2 4 8)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ns = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
    for n in ns:
        args = argparse.Namespace(gpus=n, no_cpu_baseline=False, workload="pxtran", extra=None, no_extra=False)
        t0 = time.time()
        r = bench.cpu_baseline_multirank(n, bench.extra_keys(n, args))
        print(json.dumps({"ranks": n, "seconds": round(time.time() - t0, 1),
                          "baselines": {k: {"value": v["value"], "cores": v["cores"], "sample": v["sample"]}
                                        for k, v in r.items()}}), flush=True)


if __name__ == "__main__":
    main()
