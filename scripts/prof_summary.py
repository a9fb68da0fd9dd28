"""Summarize a rocprofv3 --kernel-trace --stats CSV directory into a markdown table."""
import csv
import glob
import os
import sys

d = sys.argv[1]
stats = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
rows = list(csv.DictReader(open(stats)))
print("| kernel | calls | avg us | total ms | % |")
print("|---|---|---|---|---|")
for r in rows:
    name = r["Name"].replace("|", "/")
    if len(name) > 90:
        name = name[:87] + "..."
    print(f"| {name} | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {float(r['TotalDurationNs'])/1e6:.3f} | {float(r['Percentage']):.1f} |")
