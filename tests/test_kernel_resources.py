"""Device code of the shipped library (no GPU): none of our kernels may use scratch (private)
memory.

A runtime-indexed register array lands in scratch; in r2 the large shape's 4 x 4 lane
transpose for 4-byte elements kept 144 bytes per lane there and ran fp32 transposes at 3.3
instead of 5.3-5.7 TB/s.  The gfx950 code objects are extracted from libcosta_amd.so and every
kernel's `.private_segment_fixed_size` is read from its metadata notes."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "costa_amd", "lib", "libcosta_amd.so")
LLVM = "/opt/rocm/lib/llvm/bin"


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(f"{LLVM}/llvm-objdump")),
                    reason="library or ROCm LLVM tools not available")
def test_no_kernel_uses_scratch(tmp_path):
    lib = tmp_path / "libcosta_amd.so"
    shutil.copy(LIB, lib)
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", str(lib)], check=True,
                   capture_output=True, cwd=tmp_path)
    objs = [p for p in tmp_path.iterdir() if "gfx950" in p.name]
    assert objs, "no gfx950 code object in libcosta_amd.so"
    kernels = {}
    for o in objs:
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(o)], check=True,
                               capture_output=True, text=True).stdout
        # each kernel's metadata block: .name ... .private_segment_fixed_size (YAML, one map each)
        for block in re.split(r"\n\s+- \.", notes):
            name = re.search(r"\.name:\s+(\S+)", block)
            size = re.search(r"\.private_segment_fixed_size:\s+(\d+)", block)
            if name and size:
                kernels[name.group(1)] = int(size.group(1))
    assert any("tile_kernel" in k for k in kernels) and any("tiny_kernel" in k for k in kernels)
    # our kernels (namespace costa); rocPRIM's radix sort used by the device planner is its own
    scratch = {k: v for k, v in kernels.items() if v and "costa" in k}
    assert not scratch, f"kernels using scratch: {scratch}"
