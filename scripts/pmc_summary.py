#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes: mean counter values per dispatch of the kernels
whose name contains the given substring, plus derived rates (clock, VALU issue share, waits).

    python scripts/pmc_summary.py gpurun_out/cutpmc1 gpurun_out/cutpmc2 --kernel dq_scan_cut
"""
import argparse
import collections
import csv
import os


def load(dirs, sub):
    vals = collections.defaultdict(list)
    durs = []
    meta = {}
    for d in dirs:
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            if sub in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
            if sub in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
                meta = {k: r.get(k) for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "VGPR_Count",
                                              "SGPR_Count", "Accum_VGPR_Count", "Scratch_Size")}
    return {k: sum(v) / len(v) for k, v in vals.items()}, durs, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    v, durs, meta = load(a.dirs, a.kernel)
    ms = sum(durs) / max(1, len(durs))
    print(f"kernel ~ {a.kernel}: {len(durs)} dispatches, mean {ms:.3f} ms; {meta}")
    for k in sorted(v):
        print(f"  {k:28s} {v[k]:.4g}")
    if "GRBM_GUI_ACTIVE" in v and ms:
        clk = v["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3)
        print(f"  effective clock            {clk / 1e9:.3f} GHz")
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        simds = 4 * a.cus
        if "SQ_INSTS_VALU" in v:
            print(f"  VALU wave-instr per SIMD-cycle {v['SQ_INSTS_VALU'] / (simds * cyc):.3f}")
        if "SQ_WAVE_CYCLES" in v:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if k in v:
                    print(f"  {k} share of wave cycles {v[k] / v['SQ_WAVE_CYCLES']:.3f}")


if __name__ == "__main__":
    main()
