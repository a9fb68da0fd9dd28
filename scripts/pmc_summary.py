"""Summarize a rocprofv3 ``--pmc`` counter_collection.csv per kernel (mean over dispatches).

    python scripts/pmc_summary.py gpurun_out/pmc1/run_counter_collection.csv [name-substring ...]
"""
import collections
import csv
import sys


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[name][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for name, cs in per.items():
        us = sum(dur[name].values()) / max(1, len(dur[name])) / 1e3
        print(f"{name[:100]}  ({len(dur[name])} dispatches, {us:.1f} us avg)")
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main()
