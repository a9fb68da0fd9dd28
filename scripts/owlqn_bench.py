"""OWLQN solve timing (L1 WLS): device vs the native host driver on the same statistics.

k <= 128: the one-wave HIP solver (``wls_qn_kernel``); up to 4608: the cooperative grid solver
(``wls_qn_grid.hip``).  Statistics from a synthetic fp64 fit of the given width."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from net.jgp.labs.sparkdq4ml_amd.models.optim import wls_owlqn_device  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.ops import device, native  # noqa: E402

CASES = os.environ.get("CASES", "1:1.0,32:0.05,64:0.02,127:0.01,256:0.01,1024:0.01,4096:0.01").split(",")
ENGINE = "hip"
for case in CASES:
    d, reg = case.split(":")
    d, reg = int(d), float(reg)
    n = max(20_000, 4 * d)
    g = torch.Generator(device="cuda").manual_seed(d)
    X = torch.randn(d, n, generator=g, device="cuda", dtype=torch.float64)
    beta = torch.randn(d, generator=g, device="cuda", dtype=torch.float64) * (
        torch.rand(d, generator=g, device="cuda") > 0.5)
    y = beta @ X + 1.0 + 0.1 * torch.randn(n, generator=g, device="cuda", dtype=torch.float64)
    flat = device.gram_stats(X, y, None, None, "fp64")
    torch.cuda.synchronize()
    args = (flat, d, True, reg, 1.0, True, True, 100, 1e-6)
    wls_owlqn_device(*args)  # warm-up (kernel load / torch caches)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    wls, _ = wls_owlqn_device(*args)
    torch.cuda.synchronize()
    dev_ms = (time.perf_counter() - t0) * 1e3
    host = flat.cpu().numpy()
    t0 = time.perf_counter()
    r = native.host().wls_fit(host, d, True, reg, 1.0, True, True, 0, 100, 1e-6, False)
    host_ms = (time.perf_counter() - t0) * 1e3
    err = float(np.max(np.abs(np.asarray(wls.coefficients) - np.asarray(r["coefficients"]))))
    print(json.dumps({"k": d + 1, "reg": reg, "engine": ("hip_one_wave" if d + 1 <= 128 else ("hip_grid" if ENGINE == "hip" else "torch_device")),
                      "device_ms": dev_ms, "host_native_ms": host_ms, "iterations_dev": len(wls.objectiveHistory),
                      "iterations_host": len(r["objective_history"]), "max_abs_coef_diff": err}), flush=True)
