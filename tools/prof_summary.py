"""Summarise a rocprofv3 kernel_stats.csv (used for profiles/*.md)."""
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(x['TotalDurationNs']) for x in r)
print(f"{'kernel':60s} {'calls':>6s} {'total ms':>9s} {'avg us':>9s} {'%':>6s}")
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs'])):
    print(f"{x['Name'][:60]:60s} {x['Calls']:>6s} {float(x['TotalDurationNs'])/1e6:9.2f} {float(x['AverageNs'])/1e3:9.2f} {100*float(x['TotalDurationNs'])/tot:6.2f}")
