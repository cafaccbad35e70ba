"""Reading the committed golden vectors (tests/golden/*.npz) and comparing buffers to them."""
from __future__ import annotations

import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name: str):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def check_case_spec(case, fx) -> None:
    spec = bytes(fx["spec"]).decode()
    assert spec == case.spec(), f"{case.name}: case definition drifted from its fixture"


def matches(fx, key: str, buf: np.ndarray) -> bool:
    """bit-exact comparison against the reference's output (raw bytes or sha256)."""
    raw = np.ascontiguousarray(buf).tobytes()
    if key in fx:
        return raw == np.ascontiguousarray(fx[key]).tobytes()
    return hashlib.sha256(raw).digest() == bytes(fx["sha_" + key])


def first_mismatch(fx, key: str, buf: np.ndarray) -> str:
    if key not in fx:
        return "(hash mismatch)"
    ref = fx[key]
    a = np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    b = np.ascontiguousarray(ref).view(np.uint8).reshape(-1)
    if a.size != b.size:
        return f"size {a.size} vs {b.size}"
    idx = np.nonzero(a != b)[0]
    E = ref.dtype.itemsize
    i = int(idx[0]) // E
    return f"{idx.size} bytes differ; first element {i}: got {buf.reshape(-1)[i]} want {ref[i]}"
