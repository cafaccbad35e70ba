#!/usr/bin/env python3
"""A/B of bench.py lines under several environment settings, alternating, each in a fresh process
(one process = one placement of the buffers; see DESIGN §5 on process-to-process spread).

    python3 tools/ab_bench.py OUT REPS 'label:ENV=V,ENV=V' ... -- <bench.py args>

Each setting runs REPS times in the order s1 s2 ... s1 s2 ...; tuning overrides need
COSTA_TUNING=1 in the setting (the library ignores them otherwise).  Prints and appends to
OUT/ab.txt one line per run: label, kernel ms (roofline.avg_launch_ms), value, verified.  A run
that fails stops the script (exit 1)."""
import json
import os
import subprocess
import sys


def main():
    out, reps = sys.argv[1], int(sys.argv[2])
    k = sys.argv.index("--")
    settings = []
    for a in sys.argv[3:k]:
        label, _, envs = a.partition(":")
        env = dict(e.split("=", 1) for e in envs.split(",") if e)
        settings.append((label, env))
    bench_args = sys.argv[k + 1:]
    os.makedirs(out, exist_ok=True)
    log = open(os.path.join(out, "ab.txt"), "a")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for r in range(reps):
        for label, env in settings:
            e = dict(os.environ, **env)
            p = subprocess.run(["timeout", "-k", "10", "300", sys.executable, os.path.join(root, "bench.py"),
                                *bench_args], capture_output=True, text=True, env=e)
            with open(os.path.join(out, f"{label}_{r}.err"), "w") as f:
                f.write(p.stderr[-20000:])
            lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
            if p.returncode != 0 or not lines:
                print(f"{label} rep {r}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(lines[-1])
            ro = d.get("roofline") or {}
            msg = (f"{label:24s} rep {r}: kernel {ro.get('avg_launch_ms')} ms  value {d.get('value')} GB/s  "
                   f"frac {ro.get('frac')}  of_ceiling {ro.get('frac_of_ceiling')}  "
                   f"ceiling {(ro.get('copy_ceiling') or {}).get('best_GBps')}  verified {d.get('verified')}")
            print(msg, flush=True)
            log.write(msg + "\n")
            log.flush()


if __name__ == "__main__":
    main()
