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
                        "COSTA_MERGE", "COSTA_TR_SIDE", "COSTA_FORCE_SQ", "COSTA_BAND_H", "COSTA_TUNING")}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env=dict(env, COSTA_MERGE="0", COSTA_CBLOCK="0", COSTA_TUNING="1"))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    # merging of ops that continue each other (on by default)
    r = subprocess.run([str(exe), "merge"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    # the default lists' sub-tiles cover their ops exactly once, whatever order the sorts left
    # (destination panels, XCD groups of the skew shape, merged ragged blocks, cfg 5)
    # and unmerged (thousands of ops per list, sorted across ops)
    clean = {k: v for k, v in os.environ.items() if not k.startswith("COSTA_")}
    for extra in ({}, {"COSTA_MERGE": "0", "COSTA_TUNING": "1"}):
        r = subprocess.run([str(exe), "cover"], capture_output=True, text=True, timeout=300,
                           env=dict(clean, **{"COSTA_CBLOCK": "0", "COSTA_TUNING": "1", **extra}))
        assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    # destination-block groups (default on): each group's ops tile its range exactly once, and
    # with the pieces cover every op of cfg 5's lists; column bands of blocks over the budget
    r = subprocess.run([str(exe), "cblock"], capture_output=True, text=True, timeout=300, env=clean)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr
    # the transposing groups' XCD chunk order is a permutation of every launch size
    r = subprocess.run([str(exe), "xcd"], capture_output=True, text=True, timeout=300, env=clean)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


TUNING = {"COSTA_TINY_SORT": "0", "COSTA_FORCE_SQ": "1", "COSTA_LARGE_SORT": "0", "COSTA_XCD_BANDS": "0",
          "COSTA_WAVE_POLICY": "1", "COSTA_MERGE": "0", "COSTA_SKEW": "0", "COSTA_TINY_LDS": "1024",
          "COSTA_TINY_COPY": "512", "COSTA_TR_SIDE": "4", "COSTA_MISALIGNED_VEC": "3",
          "COSTA_SKEW_XCD": "2", "COSTA_CBLOCK": "0", "COSTA_CB_BANDS": "0", "COSTA_COPY_GRANULE": "0",
          "COSTA_CB_CHUNK": "16"}


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_tuning_overrides_ignored_without_opt_in(tmp_path):
    """the library must not let a user's environment pick work-list orders and shapes
    the GPU tests never run.  Every tuning override set, without COSTA_TUNING=1: the work lists of
    cfg 5 'N' / 'T', cfg 2, cfg 4, merging 24^2 blocks and lld 4097 are byte-identical to the
    default build's; with COSTA_TUNING=1 the same overrides do change them."""
    if not os.path.exists(os.path.join(LIB, "libcosta_amd.so")):
        pytest.skip("libcosta_amd.so not built (run __graft_entry__.build())")
    exe = tmp_path / "work_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "costa_amd", "csrc"),
                    os.path.join(ROOT, "tools", "work_check.cpp"), "-L" + LIB, "-lcosta_amd",
                    "-Wl,-rpath," + LIB, "-o", str(exe)], check=True, timeout=300)
    base = {k: v for k, v in os.environ.items() if not k.startswith("COSTA_")}

    def digest(env):
        r = subprocess.run([str(exe), "digest"], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        return r.stdout.strip()

    default = digest(base)
    assert default.startswith("digest ")
    assert digest(dict(base, **TUNING)) == default
    assert digest(dict(base, COSTA_TUNING="0", **TUNING)) == default
    assert digest(dict(base, COSTA_TUNING="1", **TUNING)) != default
