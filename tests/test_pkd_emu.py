"""The photon kd-tree build kernels (libyafaray_amd/csrc/pkd_kernels.h) executed on CPU threads.

tools/pkd_emu.cc compiles the same kernel source with a small emulation of the HIP execution
model (one std::thread per lane, std::barrier for __syncthreads, block-wide ballots) and checks the
tree node for node against a direct restatement of the reference build (pkdtree.h:115-222), with
every index range-checked (PKD_CHECK).  The GPU run of the same check is tools/pkd_check.py; the
photon-map parity tests (test_gpu_parity.py) cover the product path end to end.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_pkd_kernels_emulated(tmp_path):
    exe = tmp_path / "pkd_emu"
    subprocess.run(["g++", "-std=c++20", "-O1", "-pthread", os.path.join(ROOT, "tools", "pkd_emu.cc"), "-o", str(exe)], check=True)
    sizes = ["1", "2", "3", "17", "64", "65", "256", "257", "1000", "3000", "9000"]
    out = subprocess.run([str(exe)] + sizes, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("OK")
