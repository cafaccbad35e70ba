"""Pins the CPU oracle (oracle/costa_oracle.c) to the REFERENCE.

* the reference's own known answers: tests/unit/test_utils.cpp (explicit expected arrays for
  copy2D.row_major, copy2D.col_major, transpose.row_to_col_major; the rand()-based
  transpose.col_to_row_major property + the reference's output hash)
* every golden case produced by running eth-cscs/COSTA itself (tests/golden/make_fixtures.py):
  oracle outputs must be bit-identical (the special-value cases included: both run on x86, so
  even generated NaNs carry the same bits);
* the oracle's complex product against GCC's own (C99 Annex G, libgcc __muldc3 / __mulsc3).
"""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle
from cases import all_cases, special_cases
from golden_io import check_case_spec, first_mismatch, load, matches

IN8x4 = np.array([9, 1, 1, -1, 7, 3, 4, -1, 5, 5, 1, -1, 9, 2, 3, -1,
                  7, 6, 5, -1, 2, 2, 4, -1, 3, 7, 4, -1, 3, 8, 1, -1], np.int32)


def kat_inputs_col_to_row():
    """in[i] = i + rand() after srand(100) (test_utils.cpp:208-225), via this host's libc"""
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(100)
    n = 500 * 1100
    r = np.array([libc.rand() for _ in range(n)], np.int64)
    return (np.arange(n, dtype=np.int64) + r).astype(np.int32)


def test_kat_copy2d_row_major():
    # test_utils.cpp:7-73 — expected result written out in the reference test
    expected = np.zeros(40, np.int32)
    for i in range(8):
        expected[i * 5:i * 5 + 3] = IN8x4[i * 4:i * 4 + 3]
    out = np.zeros(40, np.int32)
    oracle.copy_and_transform(oracle.INT32, 8, 3, IN8x4, 4, False, out, 5, False)
    fx = load("kat")
    ref = fx["copy2D_row_major_out"]
    for i in range(8):
        assert (out[i * 5:i * 5 + 3] == expected[i * 5:i * 5 + 3]).all()
    assert (out == ref).all()


def test_kat_copy2d_col_major():
    out = np.zeros(40, np.int32)
    oracle.copy_and_transform(oracle.INT32, 3, 8, IN8x4, 4, True, out, 5, True)
    assert (out == load("kat")["copy2D_col_major_out"]).all()


def test_kat_row_to_col_major():
    # test_utils.cpp:143-206: explicit expected matrix
    expected = np.array([9, 7, 5, 9, 7, 2, 3, 3, -1, -1,
                         1, 3, 5, 2, 6, 2, 7, 8, -1, -1,
                         1, 4, 1, 3, 5, 4, 4, 1, -1, -1], np.int32)
    out = np.zeros(30, np.int32)
    oracle.copy_and_transform(oracle.INT32, 8, 3, IN8x4, 4, False, out, 10, True)
    for j in range(3):
        for i in range(8):
            assert out[j * 10 + i] == expected[j * 10 + i]
    assert (out == load("kat")["row_to_col_major_out"]).all()


def test_kat_col_to_row_major():
    fx = load("kat")
    inp = kat_inputs_col_to_row()
    assert hashlib.sha256(inp.tobytes()).digest() == bytes(fx["sha_col_to_row_major_in"])
    out = np.zeros(1000 * 501, np.int32)
    oracle.copy_and_transform(oracle.INT32, 1000, 500, inp, 1100, True, out, 501, False)
    o = out.reshape(1000, 501)[:, :500]
    i = inp.reshape(500, 1100)[:, :1000]
    assert (o == i.T).all()  # the reference's own check, test_utils.cpp:262-269
    assert hashlib.sha256(out.tobytes()).digest() == bytes(fx["sha_col_to_row_major_out"])


@pytest.mark.parametrize("case", all_cases() + special_cases(), ids=lambda c: c.name)
def test_oracle_matches_reference(case):
    fx = load(case.name)
    check_case_spec(case, fx)
    got = case.expected()
    for p in range(len(case.pairs)):
        for r in range(case.P):
            key = f"C{p}_r{r}"
            assert matches(fx, key, got[p][r]), f"{case.name} {key}: " + first_mismatch(
                fx, key, got[p][r])


SPECIAL_D = [0.0, -0.0, 1.0, -1.0, 0.5, -3.0, 1e308, -1e308, 1e-310, float("inf"), float("-inf"),
             float("nan"), -float("nan"), 2.5]
SPECIAL_F = [0.0, -0.0, 1.0, -1.0, 0.5, -3.0, 3e38, -3e38, 1e-40, float("inf"), float("-inf"),
             float("nan"), -float("nan"), 2.5]


@pytest.fixture(scope="module")
def native_cmul(tmp_path_factory):
    """GCC's own complex product (the one std::complex<T>::operator* compiles to in the
    reference's binary: naive product + __muldc3 / __mulsc3 when both parts are NaN)"""
    import subprocess
    d = tmp_path_factory.mktemp("cmul")
    src = d / "cmul.c"
    src.write_text("""
#include <complex.h>
void native_cmul(int t, const void* a, const void* b, void* out) {
    if (t == 2) *(float _Complex*)out = *(const float _Complex*)a * *(const float _Complex*)b;
    else *(double _Complex*)out = *(const double _Complex*)a * *(const double _Complex*)b;
}
""")
    so = d / "libcmul.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", str(src), "-o", str(so)],
                   check=True)
    L = ctypes.CDLL(str(so))
    L.native_cmul.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return L.native_cmul


@pytest.mark.parametrize("code", [oracle.CFLOAT, oracle.CDOUBLE])
def test_complex_product_is_gccs(native_cmul, code):
    """the oracle's restated Annex G product == GCC's, bit for bit, over every combination of
    special parts (inf, NaN, signed zeros, overflowing and subnormal values)"""
    vals = SPECIAL_F if code == oracle.CFLOAT else SPECIAL_D
    dt = np.complex64 if code == oracle.CFLOAT else np.complex128
    rt = np.float32 if code == oracle.CFLOAT else np.float64
    L = oracle.lib()
    bad = 0
    with np.errstate(all="ignore"):
        for ar in vals:
            for ai in vals:
                a = np.array([ar, ai], rt)
                for br in vals:
                    for bi in vals:
                        b = np.array([br, bi], rt)
                        got, want = np.zeros(2, rt), np.zeros(2, rt)
                        L.oracle_cmul(code, a.ctypes.data, b.ctypes.data, got.ctypes.data)
                        native_cmul(code, a.ctypes.data, b.ctypes.data, want.ctypes.data)
                        bad += got.tobytes() != want.tobytes()
    assert bad == 0, f"{bad} products differ from GCC's"


def test_special_cases_exercise_the_recovery():
    """the special-value fixtures hold products the naive formula gets wrong: infinities where
    (ac - bd, ad + bc) gives NaN in both parts"""
    case = [c for c in special_cases() if c.name == "specials_z_T"][0]
    a, _ = case.inputs(0, 0)
    out = load(case.name)["C0_r0"]
    with np.errstate(all="ignore"):
        naive_nan = np.isnan(a.real * 1.0 - a.imag * 0.0) & np.isnan(a.real * 0.0 + a.imag * 1.0)
    assert naive_nan.sum() > 20
    assert np.isinf(out.real).sum() + np.isinf(out.imag).sum() > 20
