"""ScaLAPACK drop-in: tests/scalapack/drop_in.c linked against libcosta_amd_prefixed_scalapack.so,
MKL ScaLAPACK/BLACS and the image's MPICH (no GPU needed to link; running needs one); and, on the
CPU with 4 MPI ranks, the shims' process mapping between different BLACS grids
(tests/scalapack/layout_check.cpp: the shim compiled with a hook that checks the layouts instead
of transforming)."""
import os
import shutil
import subprocess

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
    local blocks are exactly the ones it owns (no GPU: the transform is replaced by the check)."""
    exe = tmp_path / "layout_check"
    mkl = [f"{CONDA}/lib/lib{x[2:]}.so" for x in MKL]
    subprocess.run(["g++", "-std=c++17", "-O1", "-DCOSTA_PREFIXED", f"-I{ROOT}/include",
                    f"-I{CONDA}/include", os.path.join(ROOT, "tests", "scalapack", "layout_check.cpp"),
                    "-o", str(exe), f"-L{LIB}", "-lcosta_amd", *mkl, f"{CONDA}/lib/libmpi.so",
                    f"-Wl,-rpath,{LIB}", f"-Wl,-rpath,/usr/lib/x86_64-linux-gnu:{CONDA}/lib"],
                   check=True, timeout=300)
    env = dict(os.environ, PATH=f"{CONDA}/bin:" + os.environ["PATH"])
    r = subprocess.run([shutil.which("mpiexec", path=env["PATH"]) or f"{CONDA}/bin/mpiexec",
                        "-n", "4", str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr
