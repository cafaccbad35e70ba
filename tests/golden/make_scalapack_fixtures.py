"""Generate tests/golden/scalapack_np{1,4}.npz from the REFERENCE's own ScaLAPACK wrappers.

oracle/_ref/ref_scalapack is tests/scalapack/shim_cases.cpp linked with the reference's
costa_p?gemr2d / costa_p?tran* (prefixed_pxgemr2d.cpp, prefixed_pxtran{,u,c}.cpp over
costa_pxgemr2d.cpp and costa_pxtran_op.cpp) and library, compiled from /root/reference by
`make -C oracle ref scalapack`, over MKL BLACS and MPICH from /opt/conda. It runs every case of
shim_cases.cpp under `mpiexec -n 1` and `-n 4` and writes each process's local C; this script
stores those buffers, byte for byte, as uint8 arrays keyed "<case>.r<rank>".

Run in the build container (needs /root/reference):  python tests/golden/make_scalapack_fixtures.py
"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CONDA = "/opt/conda"


def main():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "scalapack"], check=True)
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_scalapack")
    env = dict(os.environ, PATH=f"{CONDA}/bin:" + os.environ["PATH"])
    for np_ in (1, 4):
        with tempfile.TemporaryDirectory() as d:
            r = subprocess.run([f"{CONDA}/bin/mpiexec", "-n", str(np_), exe, "gen", d],
                               capture_output=True, text=True, env=env, timeout=600)
            assert r.returncode == 0 and "ALL PASSED" in r.stdout, r.stdout + r.stderr
            arrays = {}
            for f in sorted(os.listdir(d)):
                assert f.endswith(".bin")
                arrays[f[:-4]] = np.fromfile(os.path.join(d, f), dtype=np.uint8)
        out = os.path.join(HERE, f"scalapack_np{np_}.npz")
        np.savez_compressed(out, **arrays)
        print(out, len(arrays), "buffers", sum(a.size for a in arrays.values()), "bytes")


if __name__ == "__main__":
    main()
