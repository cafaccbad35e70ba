"""CPU: the host planner and the layout builders under AddressSanitizer + UndefinedBehaviorSanitizer
(tests/sanitize/plan_sanitize.cpp): block-cyclic and custom layouts, every rank of 1-4 rank jobs
planned and its pack / local / unpack op lists executed on the host with an emulated exchange;
any out-of-bounds op aborts, every element of C must equal op(A) with alpha / beta exactly."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_planner_under_sanitizers(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = tmp_path / "plan_sanitize"
    csrc = os.path.join(ROOT, "costa_amd", "csrc")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-static-libasan",
           "-ffp-contract=off", "-pthread", f"-I{ROOT}/include",
           os.path.join(ROOT, "tests", "sanitize", "plan_sanitize.cpp"),
           os.path.join(csrc, "plan.cpp"), os.path.join(csrc, "layout.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip().startswith("OK"), r.stdout + r.stderr
