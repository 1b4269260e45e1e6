"""VGPR / SGPR / scratch / LDS of the kernels in a built library (or object): the gfx950 code object is
taken out of the .hip_fatbin section and its AMDGPU metadata printed.
   python tools/kernel_regs.py libyafaray_amd/libyafaray4.so [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def code_object(path, tmp):
    fat = os.path.join(tmp, "fatbin")
    subprocess.run([f"{B}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", path, os.path.join(tmp, "junk")], check=True)
    lst = subprocess.run([f"{B}/clang-offload-bundler", "--list", "--type=o", f"--input={fat}"], capture_output=True, text=True).stdout.split()
    tgt = [t for t in lst if "gfx950" in t][0]
    co = os.path.join(tmp, "co")
    subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}", f"--targets={tgt}", f"--output={co}"], check=True)
    return co


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    with tempfile.TemporaryDirectory() as tmp:
        notes = subprocess.run([f"{B}/llvm-readelf", "--notes", code_object(path, tmp)], capture_output=True, text=True).stdout
    for blk in re.split(r"\n  - \.agpr_count:", notes)[1:]:
        blk = ".agpr_count:" + blk
        g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
        name = g("name")
        if pats and not any(p in name for p in pats):
            continue
        print(f"{name[:70]:70s} vgpr {g('vgpr_count'):>4s} agpr {g('agpr_count'):>4s} sgpr {g('sgpr_count'):>4s} "
              f"scratch {g('private_segment_fixed_size'):>5s} lds {g('group_segment_fixed_size'):>5s} spill {g('vgpr_spill_count')}")


if __name__ == "__main__":
    main()
