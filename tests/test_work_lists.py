"""Work lists (engine.cpp build_work) on the CPU: BASELINE cfg 5's geometry ('N' copy list, 'T'
transposing list, and a sparse sub-list like one exchange round's), and unaligned large ops
(fp32, lld % 4 != 0) below and above the wavefront cap.  Every piece within the budget the
library uses, the pieces of each op inside it and adding up to it, in destination-address
order, large-shape ops whole and in hint order, two
builds identical (the cut runs on several host threads).  The checks live in
tools/work_check.cpp, built here with g++ against the in-tree libcosta_amd.so; block addresses
are never dereferenced."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "costa_amd", "lib")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_work_lists_cfg5(tmp_path):
    if not os.path.exists(os.path.join(LIB, "libcosta_amd.so")):
        pytest.skip("libcosta_amd.so not built (run __graft_entry__.build())")
    exe = tmp_path / "work_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "costa_amd", "csrc"),
                    os.path.join(ROOT, "tools", "work_check.cpp"), "-L" + LIB, "-lcosta_amd",
                    "-Wl,-rpath," + LIB, "-o", str(exe)], check=True, timeout=300)
    # the library's tuning overrides would change the classification the checker expects
    env = {k: v for k, v in os.environ.items()
           if k not in ("COSTA_WAVE_POLICY", "COSTA_TINY_SORT", "COSTA_LARGE_SORT", "COSTA_XCD_BANDS",
                        "COSTA_SKEW_XCD", "COSTA_TINY_LDS", "COSTA_TINY_COPY", "COSTA_MISALIGNED_VEC", "COSTA_SKEW",
                        "COSTA_MERGE", "COSTA_TR_SIDE")}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env=dict(env, COSTA_MERGE="0"))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    # merging of ops that continue each other (on by default)
    r = subprocess.run([str(exe), "merge"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
