"""Energy per config-5 fit on one MI355X: the wide fp8 SYRK + fold (``device.gram_stats`` on a
``TiledWide``, the fit's statistics pass) timed over back-to-back repetitions while a host thread
samples the board's hwmon power and sclk.  Prints one JSON line: ms per pass, board W, J per
pass, MHz.

    N=1e7 D=4096 REPS=20 python scripts/wide_energy.py
"""
import glob
import json
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd.ops import device, native  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops.layout import TiledWide  # noqa: E402


def hwmon_dir():
    """hwmon directory of the visible GPU (its PCI address), else the first card with a power file."""
    pr = torch.cuda.get_device_properties(0)
    pats = []
    if hasattr(pr, "pci_bus_id"):
        pats.append(f"/sys/bus/pci/devices/{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0/hwmon/hwmon*")
    pats.append("/sys/class/drm/card*/device/hwmon/hwmon*")
    for p in pats:
        for d in sorted(glob.glob(p)):
            if os.path.exists(os.path.join(d, "power1_average")) or os.path.exists(os.path.join(d, "power1_input")):
                return d
    return None


class Sampler:
    def __init__(self, d):
        self.d, self.w, self.f, self._run = d, [], [], False

    def _read(self, name):
        try:
            with open(os.path.join(self.d, name)) as fh:
                return float(fh.read().split()[0])
        except (OSError, ValueError, IndexError):
            return None

    def _loop(self):
        while self._run:
            p = self._read("power1_average")
            if p is None:
                p = self._read("power1_input")
            f = self._read("freq1_input")
            if p is not None:
                self.w.append(p * 1e-6)
            if f is not None:
                self.f.append(f * 1e-6)
            time.sleep(0.02)

    def __enter__(self):
        self._run = True
        self.t = threading.Thread(target=self._loop, daemon=True)
        self.t.start()
        return self

    def __exit__(self, *a):
        self._run = False
        self.t.join()

    @staticmethod
    def mid(v):
        if not v:
            return None
        a, b = len(v) // 10, len(v) - len(v) // 10
        v = v[a:b] or v
        return sum(v) / len(v)


def main():
    n = int(float(os.environ.get("N", "1e7")))
    d = int(os.environ.get("D", "4096"))
    reps = int(os.environ.get("REPS", "20"))
    if os.environ.get("LONG_MAX"):  # (A/B) the long-unit threshold, supersteps per row range
        device._LONG_UNIT_MAX_SUP = int(os.environ["LONG_MAX"])
    h = native.hip()
    eb = 8
    buf = torch.empty(int(h.wide_tiled_bytes(eb, d, n)), dtype=torch.uint8, device="cuda")
    per_row = buf.numel() // (((n + 63) // 64) * 64)
    scale = torch.full((d,), 4.5 / 448.0, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    chunk = max(64, (int(2e8) // d) // 64 * 64)
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        xc = torch.randn(d, r1 - r0, generator=g, device="cuda")
        lo = r0 * per_row
        device.pack_wide([xc], eb, None, inv_scale=1.0 / scale, out=buf[lo:lo + ((r1 - r0 + 63) // 64) * 64 * per_row],
                         shift=None)
        del xc
    T = TiledWide(buf, d, n, eb, scale)
    y = torch.randn(n, generator=g, device="cuda")
    for _ in range(3):
        device.gram_stats(T, y, None, None, "fp8")
    torch.cuda.synchronize()
    hw = hwmon_dir()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    time.sleep(0.5)
    smp = Sampler(hw) if hw else None
    if smp:
        smp.__enter__()
    e0.record()
    for _ in range(reps):
        device.gram_stats(T, y, None, None, "fp8")
    e1.record()
    e1.synchronize()
    if smp:
        smp.__exit__()
    ms = e0.elapsed_time(e1) / reps
    bar = getattr(device, "_last_gang_bar", None)
    bar_off = None if bar is None else [int(v) for v in bar.view(8, 32)[:, 1].cpu()]
    w = Sampler.mid(smp.w) if smp else None
    print(json.dumps({"rows": n, "features": d, "reps": reps, "ms_per_pass": round(ms, 3),
                      "board_w": None if w is None else round(w, 1),
                      "j_per_pass": None if w is None else round(w * ms * 1e-3, 2),
                      "sclk_mhz": None if not smp or not smp.f else round(Sampler.mid(smp.f)),
                      "samples": len(smp.w) if smp else 0, "hwmon": hw, "gang_barrier_off": bar_off}))


if __name__ == "__main__":
    main()
