"""Per-kernel HBM traffic and SQ counters of one bench frame from rocprofv3 --pmc passes.

    python tools/pmc_aggregate.py CONFIG OUT.json DIR [DIR ...]

Each DIR holds one pass's *counter_collection.csv (tools/pmc_all.sh: FETCH_SIZE, WRITE_SIZE and
three SQ groups in separate runs, no trace domains).  Dispatches are grouped by kernel kind (the
names yafaray_amd_getKernelTimes reports; every kernel of the photon kd-tree build counts as
pkd_build).  MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reads
half the bytes of a wide coalesced load.  Read bytes come from the L2's fabric read requests by size
(pass R: TCC_EA0_RDREQ_32B / _64B / _128B, 32 / 64 / 128 B each) when that pass ran — calibrated on
known byte counts by tools/pmc_probe.hip (profiles/pmc_calibration.json: streaming 16-B loads and
128-B node reads are 128-B requests, a scattered 16-B load is one 64-B request) — else FETCH_SIZE x 2
(exact only for wide streaming reads).  Output per kind: dispatches, read / write / total bytes per
launch, the raw FETCH_SIZE bytes, the request mix, and the SQ ratios (VALU lane utilisation, wait
fractions).  Infinity-Cache (MALL) hits are fabric requests too: the read bytes are L2-miss bytes,
an upper bound of the HBM bytes.
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
    if base == "k_rad_refl":
        return "k_pregather"   # one launch record of the pre-gather kind (render.cc KK_PREGATHER)
    if base in ("k_fg_first", "k_fg_long", "k_fg_sum"):
        return "k_fg"          # the per-path final gathering: one launch record per batch (render.cc KK_FG)
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
           "method": "rocprofv3 --pmc, one counter group per run (FETCH_SIZE | WRITE_SIZE | TCC_EA0_RDREQ_32B/64B/128B | SQ "
                     "groups), one frame; read bytes = 32 / 64 / 128 B per fabric read request by size (FETCH_SIZE x2 where "
                     "the request pass is missing), KB -> B; per launch = sum / dispatches",
           "kernels": {}}
    for k, v in sorted(vals.items()):
        e = {}
        nf = len(disp[k].get("FETCH_SIZE", ())) or None
        nw = len(disp[k].get("WRITE_SIZE", ())) or None
        nr = len(disp[k].get("TCC_EA0_RDREQ_128B_sum", ())) or None
        read_total = None
        if nf:
            e["dispatches"] = nf
            e["fetch_size_bytes_per_launch"] = round(1024.0 * v["FETCH_SIZE"] / nf)
            read_total, nread = 2.0 * 1024.0 * v["FETCH_SIZE"], nf
            e["read_bytes_source"] = "FETCH_SIZE x2"
        if nr:
            r32, r64, r128 = (v.get(f"TCC_EA0_RDREQ_{b}B_sum", 0.0) for b in (32, 64, 128))
            read_total, nread = 32.0 * r32 + 64.0 * r64 + 128.0 * r128, nr
            e["dispatches"] = e.get("dispatches", nr)
            e["read_bytes_source"] = "TCC_EA0_RDREQ by size"
            tot = max(1.0, r32 + r64 + r128)
            e["read_requests_per_launch"] = {"32B": round(r32 / nr), "64B": round(r64 / nr), "128B": round(r128 / nr)}
            e["read_request_mix"] = {"32B": round(r32 / tot, 4), "64B": round(r64 / tot, 4), "128B": round(r128 / tot, 4)}
        if read_total is not None:
            e["read_bytes_per_launch"] = round(read_total / nread)
        if nw:
            e["write_bytes_per_launch"] = round(1024.0 * v["WRITE_SIZE"] / nw)
        if read_total is not None and nw:
            e["hbm_bytes_per_launch"] = e["read_bytes_per_launch"] + e["write_bytes_per_launch"]
            e["hbm_bytes_total"] = round(read_total + 1024.0 * v["WRITE_SIZE"])
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
