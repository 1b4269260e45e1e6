"""GPU BVH layouts on CPU (libyafaray_amd/csrc/bvh.cc): BVH2 and BVH4 built over random triangle
soups enclose every triangle exactly once, and the device traversal order (replicated on the host
in tests/bvh_check.cc) returns the exhaustive closest / any hit within the builder's stack bound."""
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "libyafaray_amd", "csrc")


def test_bvh_layouts_match_exhaustive_hits():
    exe = os.path.join(tempfile.gettempdir(), "yaf_bvh_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(HERE, "bvh_check.cc"),
                    os.path.join(CSRC, "bvh.cc"), "-lpthread"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
