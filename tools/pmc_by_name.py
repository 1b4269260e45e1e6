"""SQ counter ratios per kernel NAME (not kind) from rocprofv3 --pmc passes (tools/pmc_kernels.sh output dirs):
    python tools/pmc_by_name.py SUBSTR DIR [DIR ...]
prints, for every kernel whose name contains SUBSTR: dispatches, VALU lane utilisation, VALU issue per
wave cycle, wait fractions, instructions per dispatch (diagnostics; bench.py uses pmc_aggregate.py)."""
import collections
import csv
import glob
import os
import sys

sub = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[2:]:
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                n = r["Kernel_Name"]
                if sub not in n:
                    continue
                k = n.split("(")[0][:70]
                vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r["Dispatch_Id"])
for k, v in vals.items():
    nd = max(1, len(disp[k]))
    out = {"dispatches": nd}
    wc = v.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in v:
                out[c.lower() + "_frac"] = round(v[c] / wc, 3)
    if v.get("SQ_ACTIVE_INST_VALU") and v.get("SQ_THREAD_CYCLES_VALU"):
        out["valu_lane_util"] = round(v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"]), 3)
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAVES", "SQ_BUSY_CYCLES",
              "SQ_WAVE_CYCLES"):
        if c in v:
            out[c.lower()] = round(v[c] / nd)
    print(k, out)
