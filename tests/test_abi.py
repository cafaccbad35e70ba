"""The C-ABI boundary: the library loads without a GPU, exports every entry point that
include/costa_hip.h declares, and reports errors through status codes (no exception crosses
the boundary)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "costa_hip.h")


def declared():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(costa_hip_\w+)\s*\(", txt)))


def test_header_declares_entry_points():
    names = declared()
    assert "costa_hip_transform" in names and "costa_hip_block_cyclic_layout" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol(costa):
    lib = ctypes.CDLL(costa.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", costa.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (costa_hip_\w+)", out))
    assert set(declared()) <= exported


def test_header_compiles_as_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "costa_hip.h"\nint main(void){costa_tile_op_t t; (void)t;'
                   ' return sizeof(costa_tile_op_t) == 40 ? 0 : 1;}\n')
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", f"-I{ROOT}/include", str(src), "-o",
                    str(exe)], check=True)
    assert subprocess.run([str(exe)]).returncode == 0


def test_status_codes_without_gpu(costa):
    """argument errors come back as COSTA_ERR_ARG with a message, never as a crash"""
    lib = costa.lib()
    out = ctypes.c_void_p()
    rc = lib.costa_hip_block_cyclic_layout(1, 10, 10, 0, 2, 1, 1, 10, 10, 1, 1, b"R", 0, 0,
                                           ctypes.c_void_p(1 << 40), 10, b"C", 0,
                                           ctypes.byref(out))
    assert rc == 1
    assert b"positive" in lib.costa_hip_last_error()
    rc = lib.costa_hip_transform(None, None, b"N", None, None, None)
    assert rc == 1


def test_cpp_api_compiles_and_plans(tmp_path, costa):
    """the C++ drop-in headers (costa/layout.hpp, costa/transform.hpp) compile against the
    library and reproduce the reference's example0 layouts (examples/example0.cpp:94-140)"""
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include <costa/layout.hpp>
#include <costa/transform.hpp>
#include <vector>
#include <cstdio>
int main() {
    std::vector<double> a(4), c(4);
    auto A = costa::block_cyclic_layout<double>(4, 4, 2, 2, 1, 1, 4, 4, 2, 2, 'R', 0, 0,
                                                a.data(), 2, 'C', 3);
    auto C = costa::block_cyclic_layout<double>(4, 4, 2, 2, 1, 1, 4, 4, 2, 2, 'C', 0, 0,
                                                c.data(), 2, 'R', 3);
    A.initialize([](int i, int j) { return double(i + j); });
    // rank 3 owns block (1, 1) in both grids
    if (A.blocks.num_blocks() != 1 || C.blocks.num_blocks() != 1) return 1;
    if (A.blocks.get_block(0).rows_interval.start != 2) return 2;
    costa::transformer<double> t(nullptr);
    t.schedule(A, C);
    try { t.transform(); } catch (const costa::hip_error& e) { std::puts(e.what()); return 0; }
    return 3;  // a null communicator must be rejected
}
''')
    exe = tmp_path / "t"
    subprocess.run(["g++", "-std=c++17", f"-I{ROOT}/include", str(src), "-o", str(exe),
                    f"-L{os.path.dirname(costa.LIB_PATH)}", "-lcosta_amd",
                    f"-Wl,-rpath,{os.path.dirname(costa.LIB_PATH)}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "null communicator" in r.stdout


def test_ceiling_library_loads_and_rejects_bad_arguments():
    """bench.py's copy-ceiling library (costa_amd/csrc/ceiling.hip): loads without a GPU, exports
    its one entry point, and refuses arguments it cannot run before touching the GPU"""
    path = os.path.join(ROOT, "costa_amd", "lib", "libcosta_ceiling.so")
    lib = ctypes.CDLL(path)
    f = lib.costa_ceiling_copy_ms
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                  ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
    ms = (ctypes.c_float * 4)()
    p = ctypes.c_void_p(1 << 40)
    assert f(1, p, p, 1 << 21, 1000, 4, ms) == -1      # column not whole 1 KiB segments
    assert f(1, p, p, 1 << 21, 1 << 20, 4, ms) == -1   # not whole 16-column groups
    assert f(2, p, p, 1000, 0, 4, ms) == -1            # not whole 16 KiB chunks
    assert f(7, p, p, 1 << 21, 0, 4, ms) == -1         # unknown kind
    assert f(0, p, p, 1 << 21, 0, 0, ms) == -1         # no repetitions
