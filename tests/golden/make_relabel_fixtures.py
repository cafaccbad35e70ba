#!/usr/bin/env python3
"""Golden outputs of the REFERENCE's rank relabelling (communication_volume +
optimal_reordering, run by oracle/_ref/ref_harness relabel) for the cases of
tests/relabel/relabel_cases.py, stored as tests/golden/relabel.json.  Only runs where
/root/reference exists (the survey container); the tests read the committed JSON.
    python tests/golden/make_relabel_fixtures.py"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests", "relabel"))

from relabel_cases import cases, spec_text  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")


def main():
    env = dict(os.environ, PATH="/opt/conda/bin:" + os.environ["PATH"], OMP_NUM_THREADS="1")
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, case in cases().items():
            spec = os.path.join(tmp, name + ".txt")
            with open(spec, "w") as f:
                f.write(spec_text(case))
            r = subprocess.run([HARNESS, "relabel", spec], capture_output=True, text=True,
                               env=env, check=True, timeout=600)
            out[name] = json.loads(r.stdout.strip().splitlines()[-1])
            print(name, out[name]["total"], out[name]["new_total"], out[name]["perm"])
    with open(os.path.join(HERE, "relabel.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
