"""FETCH_SIZE against known byte counts (tools/pmc_probe.hip): the factor that turns the counter into
bytes for each access shape.  python tools/pmc_calib.py out.json <rocprofv3 dirs...>; each dir's
<name>.log holds the probe's {"kernel", "known_bytes"} line."""
import csv
import glob
import json
import os
import sys


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    res = {"method": "rocprofv3 --pmc FETCH_SIZE (KB), then TCC_EA0_RDREQ_32B/64B/128B, per probe kernel, one run each; "
                     "4 GiB buffer, every 128-B line read at most once (HBM, past the Infinity Cache); factor = known bytes / "
                     "(FETCH_SIZE x 1024); request_bytes = 32 / 64 / 128 B per request by size",
           "patterns": {}}
    for d in dirs:
        name = os.path.basename(d).replace("pmcprobe_", "")
        known = None
        with open(d + ".log") as fh:
            for line in fh:
                if line.startswith("{") and '"known_bytes"' in line:
                    known = json.loads(line)["known_bytes"]
        fetch = 0.0
        req = {32: 0.0, 64: 0.0, 128: 0.0}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if name not in r["Kernel_Name"]:
                        continue
                    if r["Counter_Name"] == "FETCH_SIZE":
                        fetch += float(r["Counter_Value"])
                    for b in req:
                        if r["Counter_Name"] == f"TCC_EA0_RDREQ_{b}B_sum":
                            req[b] += float(r["Counter_Value"])
        fb = fetch * 1024.0
        rb = sum(b * n for b, n in req.items())
        res["patterns"][name] = {"known_bytes": known, "fetch_size_bytes": round(fb),
                                 "factor": round(known / fb, 4) if fb and known else None,
                                 "read_requests": {f"{b}B": round(n) for b, n in req.items()},
                                 "request_bytes": round(rb),
                                 "request_bytes_over_known": round(rb / known, 4) if rb and known else None}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
