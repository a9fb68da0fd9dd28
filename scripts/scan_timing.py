"""Host-side timing of one device CSV scan's phases (debug aid for csvscan._scan_chunk).

    python scripts/scan_timing.py [rows]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from benchmarks.bench_csv_pipeline import synth_csv  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops import csvscan, native  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops.device import _h2d  # noqa: E402


def main():
    rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else int(1e8)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"dq4ml_synth_{rows}.csv")
    if not os.path.exists(path):
        synth_csv(path, rows)
    data = np.fromfile(path, dtype=np.uint8)
    dev = torch.device("cuda")
    buf = torch.from_numpy(data).to(dev)
    h = native.hip()
    n, ncols, sep = buf.numel(), 2, ","
    stream = torch.cuda.current_stream(dev).cuda_stream
    acc = {}

    def t(k, t0):
        t1 = time.perf_counter()
        acc[k] = acc.get(k, 0.0) + (t1 - t0)
        return t1

    reps = 30
    for it in range(reps + 3):
        if it == 3:
            acc.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nb = int(h.csv_count_blocks(n))
        counts = torch.empty(nb + 1, dtype=torch.int64, device=dev)
        t0 = t("alloc counts", t0)
        h.csv_line_ends(buf.data_ptr(), n, counts.data_ptr(), 0, stream)
        t0 = t("launch count", t0)
        nterm = int(counts[nb].item())
        t0 = t("sync count (.item)", t0)
        nlines = nterm + 1
        ends = torch.empty(nlines, dtype=torch.int32 if h.csv_ends_i32(n) else torch.int64, device=dev)
        t0 = t("alloc ends", t0)
        h.csv_line_ends(buf.data_ptr(), n, counts.data_ptr(), ends.data_ptr(), stream)
        t0 = t("launch ends", t0)
        ends[nterm:].fill_(n)
        t0 = t("ends[nterm] = n", t0)
        dcols = [torch.empty(nlines, dtype=dt, device=dev) for dt in (torch.int32, torch.float64)]
        t0 = t("alloc cols", t0)
        ptrs = _h2d(np.array([x.data_ptr() for x in dcols] + [1, 0], dtype=np.int64), dev)
        t0 = t("_h2d ptrs", t0)
        valid = torch.empty(ncols, nlines, dtype=torch.bool, device=dev)
        keep = torch.empty(nlines, dtype=torch.bool, device=dev)
        stats = torch.zeros(2 + 2 * ncols, dtype=torch.int64, device=dev)
        t0 = t("alloc valid/keep/stats", t0)
        h.csv_parse(buf.data_ptr(), n, ends.data_ptr(), nlines, ncols, ord(sep), ptrs.data_ptr(), valid.data_ptr(),
                    keep.data_ptr(), stats.data_ptr(), stream)
        t0 = t("launch parse", t0)
        st = torch.stack([stats]).cpu().numpy()
        t0 = t("sync stats (.cpu)", t0)
        _ = st
    for k, v in acc.items():
        print(f"{k:28s} {v / reps * 1e6:9.1f} us")
    _ = csvscan


if __name__ == "__main__":
    main()
