"""K5-wide microbench (BASELINE config 5: 1e7 rows x 4096 features, fp8): stream-ingest a synthetic
matrix into the wide fragment layout in 64-row-aligned chunks, then time the LDS-tiled MFMA SYRK
(``device.gram_stats`` on a ``TiledWide``) end to end (SYRK + split-K f64 reduction)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd.ops import device, native  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops.layout import TiledWide  # noqa: E402

n = int(float(os.environ.get("N", "1e7")))
d = int(os.environ.get("D", "4096"))
eb = int(os.environ.get("EB", "8"))
reps = int(os.environ.get("REPS", "5"))
chunk = int(float(os.environ.get("CHUNK", "5e5"))) // 64 * 64
h = native.hip()
nbytes = int(h.wide_tiled_bytes(eb, d, n))
buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
per_row = nbytes // (((n + 63) // 64) * 64)
scale = torch.full((d,), 4.5 / 448.0, device="cuda")  # N(0,1) data: |x| <= 4.5 covers it
inv = 1.0 / scale
g = torch.Generator(device="cuda").manual_seed(0)
for r0 in range(0, n, chunk):
    r1 = min(n, r0 + chunk)
    Xc = torch.randn(d, r1 - r0, generator=g, device="cuda").to(torch.bfloat16)
    lo = r0 * per_row
    hi = lo + ((r1 - r0 + 63) // 64) * 64 * per_row
    device.pack_wide([Xc], eb, None, inv_scale=inv if eb == 8 else None, out=buf[lo:hi], shift=None)
    del Xc
T = TiledWide(buf, d, n, eb, scale if eb == 8 else None)
y = torch.randn(n, generator=g, device="cuda")
comp = "fp8" if eb == 8 else "bf16"
# A/B variants interleaved in one process: "ring:order:waves" (env DQ4ML_WIDE_RING/_ORDER/_WAVES)
variants = os.environ.get("VARIANTS", "5:morton:8:gang").split(",")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
res = {v: [] for v in variants}
outs = {}
for _ in range(reps):
    for v in variants:
        fields = v.split(":")
        os.environ.pop("DQ4ML_WIDE_GANG_SYNC", None)
        if fields[-1] == "nosync":
            os.environ["DQ4ML_WIDE_GANG_SYNC"] = "0"
            fields = fields[:-1]
        same = fields[-1] == "same"
        if same:
            fields = fields[:-1]
        os.environ.pop("DQ4ML_WIDE_SAMEPAIR", None)
        if same:
            os.environ["DQ4ML_WIDE_SAMEPAIR"] = "1"
        sched = "grid"
        if fields[-1] in ("gang", "gangx"):  # ...:gang = static equal-cost XCD gang, :gangx = XCD-keyed
            sched = fields[-1]
            fields = fields[:-1]
        elif fields[-1].startswith("q"):  # ...:q<h> = persistent XCD-grouped queue schedule, h row ranges/group
            sched, hq = "queue", fields[-1][1:]
            fields = fields[:-1]
            os.environ["DQ4ML_WIDE_H"] = hq
        os.environ["DQ4ML_WIDE_SCHED"] = sched
        ring, order, waves, splitk = (fields + ["8", "0"][len(fields) - 2:])[:4]
        os.environ["DQ4ML_WIDE_RING"], os.environ["DQ4ML_WIDE_ORDER"] = ring, order
        os.environ["DQ4ML_WIDE_WAVES"], os.environ["DQ4ML_WIDE_SPLITK"] = waves, splitk
        if v not in outs:  # warm-up + result
            outs[v] = device.gram_stats(T, y, None, None, comp, x_zero_dead=True)
        torch.cuda.synchronize()
        e0.record()
        out = device.gram_stats(T, y, None, None, comp, x_zero_dead=True)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1))
base = outs[variants[0]]
for v in variants:
    t = sorted(res[v])
    diff = float((outs[v] - base).abs().max() / base.abs().max())
    print(json.dumps({"variant": v, "ms_median": t[len(t) // 2], "ms_min": t[0], "max_rel_diff_vs_first": diff}))
times = sorted(res[variants[0]])
out = outs[variants[0]]
ms = times[len(times) // 2]
P = (d + 255) // 256
mfma_flops = 2.0 * n * 256 * 256 * (P * (P + 1) // 2)  # executed on the real panel pairs
useful = 1.0 * n * d * (d + 1)  # upper triangle incl. diagonal, 2 flops per MAC
diag = out[5 + 2 * d:].cpu()
jj = torch.arange(d)
dvals = diag[jj * (jj + 1) // 2 + jj]
print(json.dumps({"n": n, "d": d, "eb": eb, "ms_median": ms, "ms_min": times[0],
                  "mfma_tflops": mfma_flops / ms / 1e9, "useful_tflops": useful / ms / 1e9,
                  "rows_per_s": n / ms * 1e3, "count": float(out[0]),
                  "diag_mean_over_n": float(dvals.mean()) / n, "bytes_x": nbytes}))
