"""Aggregate rocprofv3 counter CSVs per kernel: python tools/pmc_report.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("yafamd::", "")
            if "rocclr" in k or "at::" in k:
                continue
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k)
    for n in sorted(v):
        print(f"   {n:26s} {v[n]:.4g}")
    wc = v.get("SQ_WAVE_CYCLES")
    if wc:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES"):
            if n in v:
                print(f"   {n}/WAVE_CYCLES = {v[n] / wc:.3f}")
    if v.get("SQ_ACTIVE_INST_VALU") and v.get("SQ_THREAD_CYCLES_VALU"):
        print(f"   VALU lane utilisation = {v['SQ_THREAD_CYCLES_VALU'] / (64 * v['SQ_ACTIVE_INST_VALU']):.3f}")
