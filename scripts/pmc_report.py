#!/usr/bin/env python3
"""Markdown row per kernel from the two rocprofv3 --pmc passes of ``scripts/pmc_suite.sh``:
dispatch time, effective clock, HBM-side bytes (FETCH_SIZE doubled: gfx950 reports half the bytes
of a wide streaming read, MI355X_MICROARCH.md §HBM), bytes per row, % of the 6.3 TB/s measured HBM
peak, L2 hit rate, MFMA busy share, VALU instructions per row.

    python scripts/pmc_report.py gpurun_out/pmc_lsq_a gpurun_out/pmc_lsq_b --kernel lsq_qn_kernel --rows 1e6
"""
import argparse
import collections
import csv
import os

HBM_PEAK = 6.3e12


def load(d, sub):
    vals = collections.defaultdict(list)
    durs = []
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if sub in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        if sub in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return {k: sum(v) / len(v) for k, v in vals.items()}, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--rows", type=float, default=0.0, help="rows one dispatch covers (bytes / row)")
    ap.add_argument("--cus", type=int, default=256)
    x = ap.parse_args()
    va, da = load(x.a, x.kernel)
    vb, db = load(x.b, x.kernel)
    t = sum(da) / max(1, len(da))
    clk = va.get("GRBM_GUI_ACTIVE", 0) / 8 / t if t else 0.0
    fetch = 2 * va.get("FETCH_SIZE", 0.0) * 1024  # KiB -> B, doubled (see module doc)
    hit, miss = vb.get("TCC_HIT_sum", 0.0), vb.get("TCC_MISS_sum", 0.0)
    cyc = va.get("GRBM_GUI_ACTIVE", 0) / 8
    out = collections.OrderedDict()
    out["kernel"] = x.kernel
    out["dispatches"] = len(da)
    out["ms"] = round(t * 1e3, 4)
    out["clock_GHz"] = round(clk / 1e9, 3)
    out["HBM_bytes"] = f"{fetch:.4g}"
    out["HBM_TB/s"] = round(fetch / t / 1e12, 3) if t else None
    out["%_of_6.3TB/s"] = round(100 * fetch / t / HBM_PEAK, 1) if t else None
    if x.rows:
        out["bytes/row"] = round(fetch / x.rows, 2)
        out["VALU_instr/row"] = round(va.get("SQ_INSTS_VALU", 0) * 64 / x.rows, 2) if "SQ_INSTS_VALU" in va else None
    out["L2_hit_%"] = round(100 * hit / (hit + miss), 1) if hit + miss else None
    out["L2_fabric_req_B"] = f"{vb.get('TCC_EA0_RDREQ_sum', 0) * 128:.4g}"
    out["L1->L2_req_B"] = f"{vb.get('TCP_TCC_READ_REQ_sum', 0) * 128:.4g}"
    if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in va:
        out["MFMA_busy_%"] = round(100 * va["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * x.cus * cyc), 1)
    if "SQ_WAVE_CYCLES" in va and "SQ_WAIT_ANY" in va:
        out["wait_any_share"] = round(va["SQ_WAIT_ANY"] / va["SQ_WAVE_CYCLES"], 3)
    print("| " + " | ".join(out.keys()) + " |")
    print("|" + "---|" * len(out))
    print("| " + " | ".join(str(v) for v in out.values()) + " |")


if __name__ == "__main__":
    main()
