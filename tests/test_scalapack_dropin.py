"""ScaLAPACK drop-in: tests/scalapack/drop_in.c linked against libcosta_amd_prefixed_scalapack.so,
MKL ScaLAPACK/BLACS and the image's MPICH (no GPU needed to link; running needs one); on the CPU
with 4 MPI ranks, the shims' process mapping between different BLACS grids
(tests/scalapack/layout_check.cpp: the shim compiled with a hook that checks the layouts instead
of transforming); and the shims against the REFERENCE's own wrappers
(tests/scalapack/shim_cases.cpp; fixtures tests/golden/scalapack_np{1,4}.npz, written by the
reference's costa_p?gemr2d / costa_p?tran* through tests/golden/make_scalapack_fixtures.py):
1 process on the GPU through the shipped library, 1 and 4 processes on the CPU through the shim
source with the oracle behind the hook."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONDA = "/opt/conda"
LIB = os.path.join(ROOT, "costa_amd", "lib")
MKL = ["-lmkl_scalapack_lp64", "-lmkl_blacs_intelmpi_lp64", "-lmkl_intel_lp64",
       "-lmkl_sequential", "-lmkl_core"]

need_mpi = pytest.mark.skipif(
    not (os.path.exists(f"{CONDA}/include/mpi.h") and os.path.exists(f"{CONDA}/lib/libmpi.so")
         and os.path.exists(os.path.join(LIB, "libcosta_amd_prefixed_scalapack.so"))),
    reason="MPICH / MKL ScaLAPACK or the shim library not available")


GOLDEN = os.path.join(ROOT, "tests", "golden")
ORACLE = os.path.join(ROOT, "oracle", "liboracle.so")
RPATH = [f"-Wl,-rpath,{LIB}", f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{CONDA}/lib"]


def mpiexec(n, *args):
    env = dict(os.environ, PATH=f"{CONDA}/bin:" + os.environ["PATH"])
    return subprocess.run([shutil.which("mpiexec", path=env["PATH"]) or f"{CONDA}/bin/mpiexec",
                           "-n", str(n), *args], capture_output=True, text=True, env=env,
                          timeout=300)


def reference_outputs(tmp_path, n):
    """the reference wrappers' local C buffers for the n-process cases, as files"""
    d = tmp_path / f"ref_np{n}"
    d.mkdir()
    with np.load(os.path.join(GOLDEN, f"scalapack_np{n}.npz")) as z:
        for k in z.files:
            z[k].tofile(d / f"{k}.bin")
    return d


def build_cases(tmp_path, hook):
    exe = tmp_path / ("shim_cases_hook" if hook else "shim_cases")
    src = os.path.join(ROOT, "tests", "scalapack", "shim_cases.cpp")
    mkl = [f"{CONDA}/lib/lib{x[2:]}.so" for x in MKL]
    if hook:  # the shim source + the oracle behind the hook, no GPU
        cmd = ["g++", "-std=c++17", "-O1", "-ffp-contract=off", "-DCOSTA_PREFIXED", "-DSHIM_HOOK",
               f"-I{ROOT}/include", f"-I{CONDA}/include", src, "-o", str(exe), f"-L{LIB}",
               "-lcosta_amd", ORACLE, *mkl, f"{CONDA}/lib/libmpi.so",
               f"-Wl,-rpath,{os.path.dirname(ORACLE)}", *RPATH]
    else:  # the shipped prefixed shim library
        cmd = ["g++", "-std=c++17", "-O1", "-ffp-contract=off", f"-I{CONDA}/include", src, "-o",
               str(exe), f"-L{LIB}", "-lcosta_amd_prefixed_scalapack", "-lcosta_amd", *mkl,
               f"{CONDA}/lib/libmpi.so", *RPATH]
    subprocess.run(cmd, check=True, timeout=300)
    return exe


def build(tmp_path):
    exe = tmp_path / "drop_in"
    cmd = ["gcc", "-std=c99", "-O2", "-ffp-contract=off", f"-I{ROOT}/include",
           f"-I{CONDA}/include", os.path.join(ROOT, "tests", "scalapack", "drop_in.c"), "-o",
           str(exe), f"-L{LIB}", "-lcosta_amd_prefixed_scalapack", "-lcosta_amd",
           f"-L{CONDA}/lib", *MKL, "-lmpi", "-lm", f"-Wl,-rpath,{LIB}",
           # the system libstdc++ must win over conda's older one (libamdhip64 needs GLIBCXX_3.4.30)
           f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{CONDA}/lib"]
    subprocess.run(cmd, check=True)
    return exe


@need_mpi
def test_dropin_links(tmp_path):
    """the prefixed shim library resolves against a real ScaLAPACK/BLACS/MPI link line"""
    assert build(tmp_path).exists()


@need_mpi
def test_plain_library_exports_reference_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only",
                          os.path.join(LIB, "libcosta_amd_scalapack.so")],
                         capture_output=True, text=True, check=True).stdout
    for base in ["psgemr2d", "pdgemr2d", "pcgemr2d", "pzgemr2d", "pstran", "pdtran", "pctranu",
                 "pztranu", "pctranc", "pztranc"]:
        for name in (base, base + "_", base + "__", base.upper()):
            assert f" T {name}\n" in out, name


@pytest.mark.gpu
@need_mpi
def test_dropin_runs_on_gpu(tmp_path):
    exe = build(tmp_path)
    env = dict(os.environ, PATH=f"{CONDA}/bin:" + os.environ["PATH"])
    r = subprocess.run([shutil.which("mpiexec", path=env["PATH"]) or f"{CONDA}/bin/mpiexec",
                        "-n", "1", str(exe)], capture_output=True, text=True, env=env,
                       timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr


@need_mpi
def test_shim_process_mapping_4_ranks(tmp_path):
    """p?gemr2d between a 2x2 grid and a 1x2 grid of two of the ranks (the other two pass
    desc[CTXT] = -1), ictxt a permuted 1x4 grid; p?tran on a permuted column-major grid: every
    block's owner is the communicator rank of the process BLACS puts it on, and every process's
    local blocks are exactly the ones it owns (no GPU: the transform is replaced by the check).
    Case 3 reuses BLACS process numbers over another system communicator between two calls of
    the same process pair: with a communicator cache keyed by context handle the two processes
    chose differently (create / reuse) and hung; the 120 s limit catches that."""
    exe = tmp_path / "layout_check"
    mkl = [f"{CONDA}/lib/lib{x[2:]}.so" for x in MKL]
    subprocess.run(["g++", "-std=c++17", "-O1", "-DCOSTA_PREFIXED", f"-I{ROOT}/include",
                    f"-I{CONDA}/include", os.path.join(ROOT, "tests", "scalapack", "layout_check.cpp"),
                    "-o", str(exe), f"-L{LIB}", "-lcosta_amd", *mkl, f"{CONDA}/lib/libmpi.so",
                    f"-Wl,-rpath,{LIB}", f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{CONDA}/lib"],
                   check=True, timeout=300)
    env = dict(os.environ, PATH=f"{CONDA}/bin:" + os.environ["PATH"])
    r = subprocess.run([shutil.which("mpiexec", path=env["PATH"]) or f"{CONDA}/bin/mpiexec",
                        "-n", "4", str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr


@need_mpi
@pytest.mark.parametrize("n", [1, 4])
def test_shims_match_reference_wrappers_cpu(tmp_path, n):
    """our shims' layouts for every case (p?gemr2d s/d/c/z, p?tran, p?tranu, p?tranc; sub-matrix
    offsets, rsrc/csrc != 0, lld > local rows, row- and column-major grids 1x1, 2x2, 1x4, 4x1;
    alpha/beta kinds incl. beta = 0 over a NaN C), executed by the oracle on the CPU: every
    process's local C equals the reference wrappers' byte for byte, lld padding included"""
    if not os.path.exists(ORACLE):
        pytest.skip("oracle/liboracle.so not built")
    exe = build_cases(tmp_path, hook=True)
    r = mpiexec(n, str(exe), "check", str(reference_outputs(tmp_path, n)))
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr


@pytest.mark.gpu
@need_mpi
def test_dropin_matches_reference_wrappers_gpu(tmp_path):
    """the shipped libcosta_amd_prefixed_scalapack.so on the GPU, one process: every 1-process
    case equals the reference wrappers' output byte for byte"""
    exe = build_cases(tmp_path, hook=False)
    r = mpiexec(1, str(exe), "check", str(reference_outputs(tmp_path, 1)))
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr
