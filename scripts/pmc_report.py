#!/usr/bin/env python3
"""Markdown row per kernel from the two rocprofv3 --pmc passes of ``scripts/pmc_suite.sh``:
dispatch time, effective clock, HBM-side bytes (FETCH_SIZE doubled: gfx950 reports half the bytes
of a wide streaming read -- the headline Gram's 6.8 GB per dispatch reads back as 3.4 GB -- see
MI355X_MICROARCH.md §HBM), bytes per row, % of the 8 TB/s HBM3E peak and of the ~6.3 TB/s a
streaming kernel sustains, L2 hit rate, fabric and L1->L2 request bytes, MFMA busy share, VALU
wave-instructions per row.

Dispatches shorter than ``--min-ms`` are left out (the data-parallel l-bfgs enqueues a few
evaluations past the end that return at once); counters and times are averaged over the same
dispatches (joined by dispatch id).

    python scripts/pmc_report.py gpurun_out/pmc_lsq_a gpurun_out/pmc_lsq_b --kernel lsq_qn_dp_pass --rows 1e6 --min-ms 1
"""
import argparse
import collections
import csv
import os

HBM_PEAK = 8.0e12
HBM_SUSTAINED = 6.3e12


def load(d, sub, min_ms):
    durs = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        if sub in r["Kernel_Name"]:
            t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            if t * 1e3 >= min_ms:
                durs[r["Dispatch_Id"]] = t
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if sub in r["Kernel_Name"] and r["Dispatch_Id"] in durs:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, list(durs.values())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--rows", type=float, default=0.0, help="rows one dispatch covers (bytes / row)")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--min-ms", type=float, default=0.0)
    x = ap.parse_args()
    va, da = load(x.a, x.kernel, x.min_ms)
    vb, db = load(x.b, x.kernel, x.min_ms)
    t = sum(da) / max(1, len(da))
    cyc = va.get("GRBM_GUI_ACTIVE", 0) / 8
    clk = cyc / t if t else 0.0
    fetch = 2 * va.get("FETCH_SIZE", 0.0) * 1024  # KiB -> B, doubled (see module doc)
    hit, miss = vb.get("TCC_HIT_sum", 0.0), vb.get("TCC_MISS_sum", 0.0)
    out = collections.OrderedDict()
    out["kernel"] = x.kernel
    out["dispatches"] = len(da)
    out["ms"] = round(t * 1e3, 4)
    out["clock_GHz"] = round(clk / 1e9, 3)
    out["HBM_bytes"] = f"{fetch:.4g}"
    out["TB/s"] = round(fetch / t / 1e12, 3) if t else None
    out["%_of_8TB/s"] = round(100 * fetch / t / HBM_PEAK, 1) if t else None
    out["%_of_6.3TB/s"] = round(100 * fetch / t / HBM_SUSTAINED, 1) if t else None
    if x.rows:
        out["bytes/row"] = round(fetch / x.rows, 2)
        if "SQ_INSTS_VALU" in va:
            out["VALU_wave_instr/row"] = round(va["SQ_INSTS_VALU"] / x.rows, 3)
    out["L2_hit_%"] = round(100 * hit / (hit + miss), 1) if hit + miss else None
    out["fabric_req_B"] = f"{vb.get('TCC_EA0_RDREQ_sum', 0) * 128:.4g}"
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
