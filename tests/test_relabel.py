"""CPU: rank relabelling (costa::communication_volume + costa::optimal_reordering through the
drop-in headers) against the reference's outputs (tests/golden/relabel.json, made by
tests/golden/make_relabel_fixtures.py from oracle/_ref/ref_harness).

* The communication graph (every rank pair's volume, local pairs included) must equal the
  reference's exactly.
* The proposed permutation must equal the reference's on every case with no tie between pair
  worths (bc_T, bc_remap, custom).  On `permuted` four pairs are worth exactly the same
  (250000 each): the reference takes them in its unordered_map's iteration order through an
  unstable std::sort (comm_volume.hpp:36-50, ranks_reordering.cpp:16-39), ours by rank ids, and
  both keep the same volume local.  On the README geometry ours must keep more data local than
  the reference's.  Known reference bug not copied: optimal_reordering reads
  volume[{a, a}] with operator[] while iterating the same unordered_map
  (ranks_reordering.cpp:18-33), which inserts keys and can invalidate the iteration, so
  candidate pairs get lost; on the README case it keeps 16.7 % where the published figure
  (README.md:461-470, "Comm volume reduction [%] = 33.3333") is what the intended algorithm
  gives.  Ours must reproduce the published 33.3333 %."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "relabel"))

from relabel_cases import cases, spec_text  # noqa: E402

GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "relabel.json")))


@pytest.fixture(scope="module")
def exe(tmp_path_factory, costa):
    out = tmp_path_factory.mktemp("relabel") / "relabel_check"
    libdir = os.path.dirname(costa.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O2", f"-I{ROOT}/include",
                    os.path.join(ROOT, "tests", "relabel", "relabel_check.cpp"), "-o", str(out),
                    f"-L{libdir}", "-lcosta_amd", f"-Wl,-rpath,{libdir}"], check=True, timeout=300)
    return out


@pytest.mark.parametrize("name", sorted(cases()))
def test_relabel_vs_reference(exe, tmp_path, name):
    case = cases()[name]
    spec = tmp_path / "spec.txt"
    spec.write_text(spec_text(case))
    r = subprocess.run([str(exe), str(spec)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got, ref = json.loads(r.stdout), GOLD[name]
    assert got["volume"] == ref["volume"]
    assert got["total"] == ref["total"]
    P = case[0]
    perm = got["perm"]
    assert sorted(perm) == list(range(P))
    assert all(perm[perm[k]] == k for k in range(P))  # pairs of swapped ranks
    if name == "readme":  # the documented divergence: the published figure, not the bug's
        assert got["perm"] != ref["perm"] and got["new_total"] < ref["new_total"]
        assert round(100.0 * (got["total"] - got["new_total"]) / got["total"], 4) == 33.3333
        assert round(100.0 * (ref["total"] - ref["new_total"]) / ref["total"], 4) == 16.6667
    elif name == "permuted":  # a tie between equal pair worths, broken differently
        assert (perm, ref["perm"]) == ([1, 0, 3, 2], [2, 3, 0, 1])
        assert got["new_total"] == ref["new_total"] == got["total"] // 2
    else:
        assert perm == ref["perm"], f"permutation differs from the reference's: {perm} vs {ref['perm']}"
        assert got["new_total"] == ref["new_total"] and got["reordered"] == ref["reordered"]
