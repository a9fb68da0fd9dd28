"""Config-5 SYRK limiter diagnosis: time AND board power per variant of the wide fp8 Gram.

Each variant (``scripts/wide_bench.py`` syntax: ``ring:order:waves[:splitk][:gang|:q<h>][:same]``)
runs back to back for ``DUR`` seconds while a thread samples the GPU's board power from hwmon
(``power1_average`` / ``power1_input``; amd-smi as a fallback).  Printed per variant: ms per
SYRK + fold, mean W, J per fit.  Ablations (timing only, wrong results): waves 81 = no MFMA,
82 = no global_load_lds after the ring prologue, ``:same`` = every block reads panels (0, 1).

    N=1e7 VARIANTS=5:morton:8:gang,5:morton:82:gang DUR=4 python scripts/wide_diag.py
"""
import glob
import json
import os
import subprocess
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd.ops import device, native  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops.layout import TiledWide  # noqa: E402


def _power_files():
    fs = []
    for pat in ("/sys/class/drm/card*/device/hwmon/hwmon*/power1_average",
                "/sys/class/drm/card*/device/hwmon/hwmon*/power1_input"):
        for f in sorted(glob.glob(pat)):
            try:
                int(open(f).read().strip())
                fs.append(f)
            except (OSError, ValueError):
                pass
    return fs


class PowerSampler:
    """Polls every readable board-power file (µW) every ``period`` s; the card under load is the
    one whose mean rises most over the idle reading."""

    def __init__(self, period=0.05):
        self.files = _power_files()
        self.period = period
        self.samples = []
        self._stop = threading.Event()
        self.idle = self._read()

    def _read(self):
        out = []
        for f in self.files:
            try:
                out.append(int(open(f).read().strip()) / 1e6)
            except (OSError, ValueError):
                out.append(float("nan"))
        if not self.files:
            try:
                r = subprocess.run(["amd-smi", "metric", "-p", "--json"], capture_output=True, text=True, timeout=5)
                js = json.loads(r.stdout)
                for g in js if isinstance(js, list) else [js]:
                    p = g.get("power", {})
                    v = p.get("socket_power", p.get("average_socket_power"))
                    if isinstance(v, dict):
                        v = v.get("value")
                    out.append(float(v))
            except Exception:  # noqa: BLE001 - diagnostic only
                pass
        return out

    def _run(self):
        while not self._stop.is_set():
            self.samples.append(self._read())
            time.sleep(self.period)

    def __enter__(self):
        self.samples = []
        self._stop.clear()
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()
        return self

    def __exit__(self, *a):
        self._stop.set()
        self.t.join()

    def mean(self):
        rows = [s for s in self.samples if s]
        if not rows:
            return None, None
        k = len(rows[0])
        means = [sum(r[i] for r in rows if i < len(r)) / len(rows) for i in range(k)]
        j = max(range(k), key=lambda i: means[i] - (self.idle[i] if i < len(self.idle) else 0.0))
        return means[j], j


def _stamp_report(h, T, y, comp, v):
    """Per-unit start / end times of every gang block (s_memrealtime, 100 MHz): how far apart the
    blocks of one XCD group run the units of one round (the same row range, sharing panels in L2)."""
    grid = device._wide_grid(h)
    st = torch.zeros(grid * 64 * 2, dtype=torch.int64, device="cuda")
    h.gram_wide_set_stamps(st.data_ptr())
    try:
        device.gram_stats(T, y, None, None, comp, x_zero_dead=True)
        torch.cuda.synchronize()
    finally:
        h.gram_wide_set_stamps(0)
    s = st.view(grid, 64, 2).cpu().double() / 100.0  # us
    t0 = s[:, 0, 0].min()
    G = grid // 8
    spreads_start, spreads_end, durs = [], [], []
    for g in range(8):
        blocks = [l * 8 + g for l in range(G)]
        for k in range(64):
            a = s[blocks, k, 0]
            b = s[blocks, k, 1]
            if bool((a == 0).any()):
                break
            spreads_start.append(float(a.max() - a.min()))
            spreads_end.append(float(b.max() - b.min()))
            durs.extend((b - a).tolist())
    import statistics as stt
    q = lambda xs, f: sorted(xs)[int(f * (len(xs) - 1))] if xs else None  # noqa: E731
    print(json.dumps({"variant": v, "rounds": len(spreads_start), "unit_us_median": round(stt.median(durs), 1),
                      "unit_us_min": round(min(durs), 1), "unit_us_max": round(max(durs), 1),
                      "round_start_spread_us_median": round(q(spreads_start, 0.5), 1),
                      "round_start_spread_us_p90": round(q(spreads_start, 0.9), 1),
                      "round_end_spread_us_median": round(q(spreads_end, 0.5), 1),
                      "first_start_spread_us": round(float(s[:, 0, 0].max() - t0), 1)}), flush=True)


def main():
    n = int(float(os.environ.get("N", "1e7")))
    d = int(os.environ.get("D", "4096"))
    eb = int(os.environ.get("EB", "8"))
    dur = float(os.environ.get("DUR", "4"))
    h = native.hip()
    nbytes = int(h.wide_tiled_bytes(eb, d, n))
    buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    per_row = nbytes // (((n + 63) // 64) * 64)
    scale = torch.full((d,), 4.5 / 448.0, device="cuda")
    chunk = 500_032
    g = torch.Generator(device="cuda").manual_seed(0)
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        Xc = torch.randn(d, r1 - r0, generator=g, device="cuda").to(torch.bfloat16)
        lo = r0 * per_row
        hi = lo + ((r1 - r0 + 63) // 64) * 64 * per_row
        device.pack_wide([Xc], eb, None, inv_scale=1.0 / scale if eb == 8 else None, out=buf[lo:hi], shift=None)
        del Xc
    T = TiledWide(buf, d, n, eb, scale if eb == 8 else None)
    y = torch.randn(n, generator=g, device="cuda")
    comp = "fp8" if eb == 8 else "bf16"
    ps = PowerSampler()
    print(json.dumps({"power_files": ps.files, "idle_W": ps.idle}))
    variants = os.environ.get("VARIANTS", "5:morton:8:gang,5:morton:82:gang,5:morton:81:gang").split(",")
    for v in variants:
        f = v.split(":")
        os.environ.pop("DQ4ML_WIDE_SAMEPAIR", None)
        os.environ.pop("DQ4ML_WIDE_GANG_SYNC", None)
        if f[-1] == "nosync":  # gang without the per-round group barrier
            os.environ["DQ4ML_WIDE_GANG_SYNC"] = "0"
            f = f[:-1]
        if f[-1] == "same":
            os.environ["DQ4ML_WIDE_SAMEPAIR"] = "1"
            f = f[:-1]
        sched = "grid"
        if f[-1] in ("gang", "gangx"):
            sched, f = f[-1], f[:-1]
        elif f[-1].startswith("q"):
            sched, os.environ["DQ4ML_WIDE_H"], f = "queue", f[-1][1:], f[:-1]
        os.environ["DQ4ML_WIDE_SCHED"] = sched
        ring, order, waves, splitk = (f + ["8", "0"][len(f) - 2:])[:4]
        os.environ["DQ4ML_WIDE_RING"], os.environ["DQ4ML_WIDE_ORDER"] = ring, order
        os.environ["DQ4ML_WIDE_WAVES"], os.environ["DQ4ML_WIDE_SPLITK"] = waves, splitk
        if sched == "gangx":
            os.environ["DQ4ML_WIDE_XCCDBG"] = "1"
        device.gram_stats(T, y, None, None, comp, x_zero_dead=True)  # warm-up
        torch.cuda.synchronize()
        os.environ.pop("DQ4ML_WIDE_XCCDBG", None)
        if sched == "gangx" and device._last_xcc is not None:
            # census: does blockIdx % 8 name the XCD (the static gang's assumption)?
            x = device._last_xcc.cpu().tolist()
            per = [x.count(i) for i in range(8)]
            rr = all(x[b] == x[b % 8] for b in range(len(x)))
            print(json.dumps({"xcc_blocks_per_xcd": per, "blockIdx_mod8_is_xcd": rr, "first16": x[:16]}))
        if os.environ.get("STAMPS") and sched == "gang" and waves == "8":
            _stamp_report(h, T, y, comp, v)
        time.sleep(1.0)  # let the board cool to the same start point for every variant
        t0 = time.perf_counter()
        k = 0
        with ps:
            while time.perf_counter() - t0 < dur:
                device.gram_stats(T, y, None, None, comp, x_zero_dead=True)
                k += 1
                if k % 4 == 0:
                    torch.cuda.synchronize()
            torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / k
        w, card = ps.mean()
        print(json.dumps({"variant": v, "fits": k, "ms_per_fit": round(ms, 3), "mean_W": w, "card": card,
                          "J_per_fit": None if w is None else round(w * ms / 1e3, 3),
                          "samples": len(ps.samples)}), flush=True)


if __name__ == "__main__":
    main()
