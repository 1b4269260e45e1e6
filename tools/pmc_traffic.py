"""HBM traffic per k_trace launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py FETCH.csv WRITE.csv CONFIG OUT.json [VALU.csv]

MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KB (x1024); on gfx950 FETCH_SIZE
reports half of the bytes of a wide coalesced read, so it is doubled here.  The result is an
average over every k_trace dispatch of the profiled run (the same launch mix as one bench step).
With a third pass (SQ_INSTS_VALU) the VALU wave-instructions per launch are recorded too: k_trace on
an LDS-resident scene is bounded by VALU issue, not HBM.
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_src_sha1():
    with open(os.path.join(ROOT, "libyafaray_amd", "csrc", "kernels.hip"), "rb") as f:
        return hashlib.sha1(f.read()).hexdigest()


def per_dispatch(path, counter, kernel="k_trace"):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter or not r["Kernel_Name"].startswith(kernel) and \
                    f" {kernel}" not in r["Kernel_Name"] and f"{kernel}<" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            if "k_trace_rays" in name:
                continue
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return vals


def main():
    fetch_csv, write_csv, config, out = sys.argv[1:5]
    valu_csv = sys.argv[5] if len(sys.argv) > 5 else None
    fe = per_dispatch(fetch_csv, "FETCH_SIZE")
    wr = per_dispatch(write_csv, "WRITE_SIZE")
    if not fe or not wr:
        sys.exit("no k_trace dispatches with the counters found")
    fetch = 2.0 * 1024.0 * sum(fe.values()) / len(fe)
    write = 1024.0 * sum(wr.values()) / len(wr)
    res = {"config": config, "kernel": "k_trace", "kernels_hip_sha1": kernel_src_sha1(), "dispatches": [len(fe), len(wr)],
           "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
           "hbm_bytes_per_launch": round(fetch + write),
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE separate passes, FETCH_SIZE x2 (gfx950), KB->B"}
    if valu_csv:
        va = per_dispatch(valu_csv, "SQ_INSTS_VALU")
        if va:
            res["valu_insts_per_launch"] = round(sum(va.values()) / len(va))
            res["method"] += "; --pmc SQ_INSTS_VALU third pass (wave-instructions)"
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
