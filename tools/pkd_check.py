"""Range-checked photon kd-tree build on the GPU against a numpy restatement of the reference's build.

Uses libyafaray_amd/pkd_check.so (`make -C libyafaray_amd/csrc pkdcheck`): pkd.hip compiled with
-DPKD_CHECK, where every computed index is checked before use and the first failure is reported
as a source line instead of a memory fault.  The numpy tree follows pkdtree.h:115-222 (median
element (start + end) / 2 of the largest bound axis, order coordinate then index).

    python tools/pkd_check.py [n ...]
"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def okey(f):
    f = np.where(f == 0, np.float32(0), f).astype(np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xffffffff, u | 0x80000000)


def largest(lo, hi):
    dx, dy, dz = (np.float32(hi[k]) - np.float32(lo[k]) for k in range(3))
    return (0 if dx > dz else 2) if dx > dy else (1 if dy > dz else 2)


def ref_tree(pos):
    n = len(pos)
    keys = [okey(pos[:, a]) for a in range(3)]
    bits = pos.view(np.uint32)
    nodes = np.zeros((2 * n - 1, 4), np.uint32)
    depth = 0
    stack = [(0, np.arange(n), pos.min(0).copy(), pos.max(0).copy(), 0)]
    while stack:
        node, idx, lo, hi, d = stack.pop()
        depth = max(depth, d)
        if len(idx) == 1:
            i = int(idx[0])
            nodes[node] = (bits[i, 0], bits[i, 1], bits[i, 2], 3 | (i << 2))
            continue
        ax = largest(lo, hi)
        o = idx[np.lexsort((idx, keys[ax][idx]))]
        h = len(idx) // 2
        sp = pos[o[h], ax]
        right = node + 2 * h
        nodes[node] = (bits[o[h], ax], 0, 0, ax | (right << 2))
        lhi = hi.copy(); lhi[ax] = sp
        rlo = lo.copy(); rlo[ax] = sp
        stack.append((node + 1, o[:h], lo, lhi, d + 1))
        stack.append((right, o[h:], rlo, hi, d + 1))
    return nodes, depth


def positions(n, rng):
    p = rng.random((n, 3), dtype=np.float32) * np.float32(4) - np.float32(2)
    if n > 10:
        p[::7, 1] = 0.5          # ties on one axis
        p[::11, 0] = -0.0        # signed zeros compare equal
        p[1::11, 0] = 0.0
        p[::13] = p[0]           # coincident photons
    return p


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "..", "libyafaray_amd", "pkd_check.so"))
    lib.yafamd_build_pkd.restype = ctypes.c_int
    lib.yafamd_build_pkd.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_void_p,
                                     ctypes.POINTER(ctypes.c_void_p)]
    lib.yafamd_pkd_check_error.restype = ctypes.c_uint32
    lib.yafamd_pkd_check_lists.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
    lib.yafamd_pkd_scratch_free.argtypes = [ctypes.c_void_p]
    scratch = ctypes.c_void_p(None)   # the build scratch (caller-owned, reused across sizes)
    sizes = [int(a) for a in sys.argv[1:]] or [1, 2, 3, 255, 256, 257, 513, 1000, 30000, 60000]
    rng = np.random.default_rng(7)
    ok = True
    for n in sizes:
        pos = positions(n, rng)
        p4 = np.zeros((n, 4), np.float32)
        p4[:, :3] = pos
        dpos = torch.from_numpy(p4).cuda()
        dnodes = torch.zeros((2 * n - 1, 4), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        depth = ctypes.c_int(0)
        rc = lib.yafamd_build_pkd(dpos.data_ptr(), n, dnodes.data_ptr(), ctypes.byref(depth), None, ctypes.byref(scratch))
        torch.cuda.synchronize()
        err = lib.yafamd_pkd_check_error()
        lists = np.zeros((3, n, 4), np.uint32)
        lib.yafamd_pkd_check_lists(scratch, lists.ctypes.data, n)
        keys = [okey(pos[:, a]) for a in range(3)]
        for a in range(3):
            o = np.lexsort((np.arange(n), keys[a]))
            if n <= 256 and not np.array_equal(lists[a][:, 3], o):
                print(f"n={n}: list {a} not in (key, index) order: {lists[a][:8, 3].tolist()} want {o[:8].tolist()}", flush=True)
            kk = np.stack([keys[0], keys[1], keys[2]], 1)[lists[a][:, 3] % n]
            if not np.array_equal(kk.astype(np.uint32), lists[a][:, :3]):
                print(f"n={n}: list {a} keys do not match their index", flush=True)
        got = dnodes.cpu().numpy().view(np.uint32)
        line = f"n={n}: rc={rc} check_line={err} depth={depth.value}"
        if rc != 0 or err != 0:
            print(line, "FAIL", flush=True)
            ok = False
            break
        if n <= 100000:
            want, wdepth = ref_tree(pos)
            bad = np.nonzero((got != want).any(1))[0]
            line += f" ref_depth={wdepth} mismatching_nodes={len(bad)}"
            if len(bad) or wdepth != depth.value:
                ok = False
                line += f" first={bad[:4].tolist()} got={got[bad[:2]].tolist()} want={want[bad[:2]].tolist()}"
        else:
            leaves = got[(got[:, 3] & 3) == 3, 3] >> 2
            line += f" leaves_perm={np.array_equal(np.sort(leaves), np.arange(n))}"
        print(line, flush=True)
    lib.yafamd_pkd_scratch_free(scratch)
    print("OK" if ok else "FAILED")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
