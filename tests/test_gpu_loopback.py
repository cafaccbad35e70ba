"""The exchange path (PACK -> RCCL group of ncclSend/ncclRecv -> UNPACK, with its streams,
events and send/recv workspaces) on ONE GPU: in COSTA_LOOPBACK=1 mode a one-rank communicator
holds a one-rank RCCL communicator and routes its own tiles through the exchange with itself
(engine.hpp loopback_exchange); mode 2 routes half of them, the rest runs through the LOCAL
launch on the second stream concurrently with the exchange, as on a multi-GPU node.  Two ranks cannot share a GPU under RCCL, so this is how the
multi-rank machinery runs on the one-GPU box; results must equal the reference's golden
outputs bit for bit.  Runs in a child process (the mode is fixed per process)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode,slot,planner", [("1", None, None), ("2", None, None),
                                               ("2", "1", None), ("1", None, "2"),
                                               ("1", None, "lists"), ("2", None, "lists")])
def test_loopback_exchange_matches_golden(mode, slot, planner):
    """slot "1": 1 MiB host pipeline slots (many groups, ops cut into pieces); planner "2": every
    plan (pack / unpack lists, package geometry) built by the device planner; "lists": that, and
    the destination-block groups of every local and unpack list built on the GPU
    (COSTA_LIST_BUILDER=2)"""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "loopback_child.py")
    env = dict(os.environ, COSTA_LOOPBACK=mode)
    if slot:
        env["COSTA_HOST_SLOT_MIB"] = slot
        env["COSTA_TUNING"] = "1"  # the slot size is a tuning override
    if planner:
        env["COSTA_PLANNER"] = "2"
    if planner == "lists":
        env["COSTA_LIST_BUILDER"] = "2"
    r = subprocess.run([sys.executable, child], env=env, capture_output=True, text=True,
                       timeout=600)
    out = r.stdout.strip().splitlines()
    assert r.returncode == 0 and out and out[-1].startswith("OK"), r.stdout + r.stderr
    host = [l for l in out if l.startswith("HOST")]
    assert host and int(host[-1].split()[1]) > 0, "pipelined host staging did not run"
    direct = [l for l in out if l.startswith("DIRECT")]
    # page-locked host cases: pack / unpack groups moved by strided DMA (one rectangle per group)
    assert direct and int(direct[-1].split()[1]) > 0, "no direct (DMA) group ran from page-locked memory"
    if planner == "lists" and mode == "1":  # (mode 2 splits a block's tiles between two lists)
        lists = [l for l in out if l.startswith("LISTS")]
        assert lists and int(lists[-1].split()[1]) > 0, "no work list built on the GPU"
    _, n, packs, unpacks, locals_ = out[-1].split()
    assert int(packs) >= int(n) and int(unpacks) >= int(n), out[-1]  # every case exchanged
    if mode == "1":
        assert int(locals_) == 0, out[-1]
    else:  # half the tiles local: the LOCAL launch overlaps the exchange
        assert int(locals_) >= int(n) // 2, out[-1]
