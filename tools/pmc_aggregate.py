"""Per-kernel HBM traffic and SQ counters of one bench frame from rocprofv3 --pmc passes.

    python tools/pmc_aggregate.py CONFIG OUT.json DIR [DIR ...]

Each DIR holds one pass's *counter_collection.csv (tools/pmc_all.sh: FETCH_SIZE, WRITE_SIZE and
three SQ groups in separate runs, no trace domains).  Dispatches are grouped by kernel kind (the
names yafaray_amd_getKernelTimes reports; every kernel of the photon kd-tree build counts as
pkd_build).  MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reads
half the bytes of a wide coalesced load, so it is doubled.  Output per kind: dispatches, read /
write / total HBM bytes per launch, and the SQ ratios (VALU lane utilisation, wait fractions).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KINDS = ["k_camera", "k_trace", "k_surface", "k_tshadow", "k_shade", "k_nee", "k_gather", "k_spawn", "k_combine", "k_film",
         "k_photon_emit", "k_photon_bounce", "k_fg", "k_pregather", "k_gather_walk"]
COMPACT = ("k_photon_count", "k_photon_scan", "k_photon_scatter")
PKD = ("k_keys", "k_records", "k_bound", "k_root", "k_level_split", "k_level_partition", "k_partition", "k_seg_of", "k_subtrees", "k_parent_planes")


def kernel_src_sha1():
    # the same key as bench.py kernels_src_sha1 (one definition: bench's)
    sys.path.insert(0, ROOT)
    import bench
    return bench.kernels_src_sha1()


def kind_of(name, photon):
    n = name.replace("void ", "")
    m = re.search(r"(k_\w+)", n)
    base = m.group(1) if m else n
    if base == "k_trace_rays":
        return "k_trace_rays"
    for k in KINDS:
        if base == k:
            return k
    if base in COMPACT:
        return "photon_compact"
    if base.startswith(PKD) or "anonymous" in n and base in PKD:
        return "pkd_build"
    if "rocprim" in n or "hipcub" in n or "cub" in n:
        return "pkd_build" if photon else "aa_next_pass"
    if base.startswith("k_aa") or "aa_" in base:
        return "aa_next_pass"
    if "rocclr" in n or "at::" in n or "elementwise" in n:
        return None
    return "other"


def main():
    config, out = sys.argv[1], sys.argv[2]
    photon = "photon" in config
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for d in sys.argv[3:]:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = kind_of(r["Kernel_Name"], photon)
                    if k is None:
                        continue
                    c = r["Counter_Name"]
                    vals[k][c] += float(r["Counter_Value"])
                    disp[k][c].add(r["Dispatch_Id"])
    res = {"config": config, "kernels_src_sha1": kernel_src_sha1(),
           "method": "rocprofv3 --pmc, one counter group per run (FETCH_SIZE | WRITE_SIZE | 3 SQ groups), one frame; "
                     "FETCH_SIZE x2 (gfx950 wide loads), KB -> B; per launch = sum / dispatches",
           "kernels": {}}
    for k, v in sorted(vals.items()):
        e = {}
        nf = len(disp[k].get("FETCH_SIZE", ())) or None
        nw = len(disp[k].get("WRITE_SIZE", ())) or None
        if nf:
            e["dispatches"] = nf
            e["read_bytes_per_launch"] = round(2.0 * 1024.0 * v["FETCH_SIZE"] / nf)
        if nw:
            e["write_bytes_per_launch"] = round(1024.0 * v["WRITE_SIZE"] / nw)
        if nf and nw:
            e["hbm_bytes_per_launch"] = e["read_bytes_per_launch"] + e["write_bytes_per_launch"]
            e["hbm_bytes_total"] = round(2.0 * 1024.0 * v["FETCH_SIZE"] + 1024.0 * v["WRITE_SIZE"])
        wc = v.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in v:
                    e[n.lower() + "_frac"] = round(v[n] / wc, 4)
        if v.get("SQ_ACTIVE_INST_VALU") and v.get("SQ_THREAD_CYCLES_VALU"):
            e["valu_lane_util"] = round(v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"]), 4)
        hit, miss = v.get("TCC_HIT_sum"), v.get("TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            e["l2_hit_rate"] = round(hit / (hit + miss), 4)
        for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAVES",
                  "SQ_LDS_BANK_CONFLICT"):
            if n in v:
                nd = len(disp[k][n]) or 1
                e[n.lower() + "_per_launch"] = round(v[n] / nd)
        res["kernels"][k] = e
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
