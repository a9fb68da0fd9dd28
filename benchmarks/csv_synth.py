"""Synthetic wide-row CSV of the BASELINE.json shapes (``n`` rows x ``d`` float features + a label),
in the reference data's dialect (headerless, CR-only row terminators, no terminator after the last
row: ``data/dataset-*.csv``).  Built with torch on any device (the bytes of 1e8 x 32
rows are ~28 GB: formatted on the GPU, streamed to the file chunk by chunk).

Row: ``x_0,...,x_{d-1},y\\r`` with x ~ N(0, 1) printed ``[-]d.dddddd`` (|x| < 10) and
y = beta . x + y0 + 0.1 eps printed ``[-]ddd.dddd`` (|y| < 1000, leading zeros dropped);
``outliers`` of the rows get |y| in [100, 1000) (the DQ range rule's prey).  The values a
correctly rounded parser reads back are exactly ``v / 1e6`` and ``w / 1e4`` of the printed
integers ``v`` / ``w`` — returned alongside for oracles.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

__all__ = ["wide_rows", "write_wide_csv", "scratch_dir"]


def _digits(v: torch.Tensor, k: int) -> torch.Tensor:
    """The k least-significant decimal digits of int64 ``v`` as ASCII, most significant first."""
    p = 10 ** torch.arange(k - 1, -1, -1, device=v.device, dtype=torch.int64)
    return ((v.unsqueeze(-1) // p) % 10 + 48).to(torch.uint8)


def wide_rows(m: int, d: int, gen: torch.Generator, device, beta: torch.Tensor, outliers: float = 0.02,
              last: bool = False, y0: float = 0.5):
    """One chunk of ``m`` rows: (bytes uint8, X [d, m] f64 as parsed, y [m] f64 as parsed)."""
    x = torch.randn(d, m, generator=gen, device=device, dtype=torch.float32).double()
    v = torch.round(x.abs() * 1e6).clamp(max=9_999_999).to(torch.int64)
    xneg = (x < 0) & (v > 0)
    xval = torch.where(xneg, -v.double(), v.double()) / 1e6
    y = beta.double() @ xval + y0 + 0.1 * torch.randn(m, generator=gen, device=device, dtype=torch.float64)
    out = torch.rand(m, generator=gen, device=device) < outliers
    mag = 100.0 + 899.0 * torch.rand(m, generator=gen, device=device, dtype=torch.float64)
    y = torch.where(out, torch.where(y < 0, -mag, mag), y)
    w = torch.round(y.abs() * 1e4).clamp(max=9_999_999).to(torch.int64)
    yneg = (y < 0) & (w > 0)
    yval = torch.where(yneg, -w.double(), w.double()) / 1e4
    # features: [m, d, 10] = sign, int digit, '.', 6 digits, ','
    xt = v.t()
    fch = torch.empty(m, d, 10, dtype=torch.uint8, device=device)
    fch[:, :, 0] = ord("-")
    fch[:, :, 1] = (xt // 1_000_000 + 48).to(torch.uint8)
    fch[:, :, 2] = ord(".")
    fch[:, :, 3:9] = _digits(xt % 1_000_000, 6)
    fch[:, :, 9] = ord(",")
    fmask = torch.ones(m, d, 10, dtype=torch.bool, device=device)
    fmask[:, :, 0] = xneg.t()
    # label: sign, up to 3 integer digits, '.', 4 digits, CR
    ip = w // 10_000
    lch = torch.empty(m, 10, dtype=torch.uint8, device=device)
    lch[:, 0] = ord("-")
    lch[:, 1:4] = _digits(ip, 3)
    lch[:, 4] = ord(".")
    lch[:, 5:9] = _digits(w % 10_000, 4)
    lch[:, 9] = 13
    lmask = torch.ones(m, 10, dtype=torch.bool, device=device)
    lmask[:, 0] = yneg
    lmask[:, 1] = ip >= 100
    lmask[:, 2] = ip >= 10
    if last:
        lmask[-1, 9] = False  # no terminator after the last row (R8)
    chars = torch.cat([fch.reshape(m, 10 * d), lch], 1)
    mask = torch.cat([fmask.reshape(m, 10 * d), lmask], 1)
    return chars[mask], xval, yval


def scratch_dir(nbytes: int) -> str:
    """/dev/shm when it has room (RAM-backed: the pinned read-back is a memcpy), else $TMPDIR."""
    import tempfile

    for cand in ("/dev/shm", os.environ.get("TMPDIR", tempfile.gettempdir())):
        try:
            st = os.statvfs(cand)
            if st.f_bavail * st.f_frsize > 1.2 * nbytes:
                return cand
        except OSError:
            continue
    return tempfile.gettempdir()


def write_wide_csv(path: str, n: int, d: int, seed: int = 11, device=None, chunk: int = 1 << 20,
                   outliers: float = 0.02, keep: bool = False, beta: Optional[torch.Tensor] = None, y0: float = 0.5):
    """Write the CSV; returns (bytes written, beta[, X f64 [d, n], y f64 [n] on the host when keep)."""
    device = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    gen = torch.Generator(device=device).manual_seed(seed)
    beta = torch.linspace(-1.0, 1.0, d, device=device) if beta is None else beta.to(device)
    xs, ys = [], []
    total = 0
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        for r0 in range(0, n, chunk):
            m = min(chunk, n - r0)
            bts, xv, yv = wide_rows(m, d, gen, device, beta, outliers, last=r0 + m >= n, y0=y0)
            f.write(bts.cpu().numpy().tobytes())
            total += int(bts.numel())
            if keep:
                xs.append(xv.cpu())
                ys.append(yv.cpu())
    os.replace(tmp, path)
    if keep:
        return total, beta.cpu(), torch.cat(xs, 1), torch.cat(ys)
    return total, beta.cpu()
