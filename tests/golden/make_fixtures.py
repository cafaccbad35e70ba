#!/usr/bin/env python3
"""Generate the golden vectors from the REFERENCE implementation.

Runs oracle/_ref/ref_harness (eth-cscs/COSTA compiled from /root/reference sources by
oracle/Makefile) under MPICH's mpiexec for every case of cases.py and the reference's own
copy_and_transform known-answer tests, and stores the outputs as small fixtures here:

  tests/golden/<case>.npz     spec text + per (pair, rank) C buffer (raw if < 64 KiB,
                               else its sha256)
  tests/golden/kat.npz        outputs of tests/unit/test_utils.cpp's four cases

Only runs where /root/reference exists (the survey container).  The GPU box only reads
the committed .npz files.
    python tests/golden/make_fixtures.py [case ...]
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from cases import all_cases, special_cases  # noqa: E402

HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
MPIEXEC = "/opt/conda/bin/mpiexec"
RAW_LIMIT = 64 * 1024
NP = {0: np.float32, 1: np.float64, 2: np.complex64, 3: np.complex128}


def run(cmd, **kw):
    env = dict(os.environ, PATH="/opt/conda/bin:" + os.environ["PATH"], OMP_NUM_THREADS="1")
    subprocess.run(cmd, check=True, env=env, **kw)


def make_case(case) -> None:
    with tempfile.TemporaryDirectory() as td:
        spec = os.path.join(td, "spec.txt")
        with open(spec, "w") as f:
            f.write(case.spec())
        run([MPIEXEC, "-n", str(case.P), HARNESS, "case", spec, td])
        out = {"spec": np.frombuffer(case.spec().encode(), np.uint8)}
        for p in range(len(case.pairs)):
            for r in range(case.P):
                raw = open(os.path.join(td, f"C{p}_rank{r}.bin"), "rb").read()
                key = f"C{p}_r{r}"
                if len(raw) <= RAW_LIMIT:
                    out[key] = np.frombuffer(raw, NP[case.dtype])
                else:
                    out["sha_" + key] = np.frombuffer(hashlib.sha256(raw).digest(), np.uint8)
        np.savez_compressed(os.path.join(HERE, case.name + ".npz"), **out)


def make_kat() -> None:
    with tempfile.TemporaryDirectory() as td:
        run([HARNESS, "kat", td])
        out = {}
        for name in ["copy2D_row_major_out", "copy2D_col_major_out", "row_to_col_major_out",
                     "in8x4"]:
            out[name] = np.fromfile(os.path.join(td, f"kat_{name}.bin"), np.int32)
        for name in ["col_to_row_major_in", "col_to_row_major_out"]:
            raw = open(os.path.join(td, f"kat_{name}.bin"), "rb").read()
            out["sha_" + name] = np.frombuffer(hashlib.sha256(raw).digest(), np.uint8)
        np.savez_compressed(os.path.join(HERE, "kat.npz"), **out)


def main(argv):
    if not os.path.exists(HARNESS):
        run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"])
    want = set(argv[1:])
    if not want or "kat" in want:
        make_kat()
    for c in all_cases() + special_cases():
        if want and c.name not in want:
            continue
        make_case(c)
        print("fixture", c.name, "P =", c.P)


if __name__ == "__main__":
    main(sys.argv)
