"""Deferred device-side assertions: data-dependent errors without a host sync.

Spark fails a job when a task hits bad data (a null handed to ``VectorAssembler`` with
``handleInvalid=error``, a null weight in ``LinearRegression.fit``).  Evaluating such a condition
eagerly costs a device->host sync per check, which serialises an otherwise asynchronous fit
(``dq4ml.fit.async``).  Instead the condition is reduced ON the device to a one-element flag and
carried with the column / the pending fit; it is read together with the first result the host
needs anyway (``show``/``collect`` rows, the fit's coefficients), where the same exception is
raised.  The same contract as ``RaiseIfNull``'s device error flag in ``ops/dqvm.py``.
"""
from __future__ import annotations

from typing import Callable, Iterable, List, Optional

import torch

__all__ = ["DeviceCheck", "defer", "verify"]


class DeviceCheck:
    """``flag`` (a one-element device tensor, nonzero = failed) plus the exception to raise."""

    __slots__ = ("flag", "make_exc")

    def __init__(self, flag: torch.Tensor, make_exc: Callable[[], BaseException]):
        self.flag, self.make_exc = flag, make_exc

    def __repr__(self):
        return f"DeviceCheck({self.flag.device})"


def defer(flag: torch.Tensor, make_exc: Callable[[], BaseException]) -> Optional[DeviceCheck]:
    """Host tensors are checked at once (no sync to save); device tensors become a pending check."""
    if not flag.is_cuda:
        if bool(flag.reshape(-1).any()):
            raise make_exc()
        return None
    # a view of the flag, kept as it is (no conversion kernel per deferred check: one per fit of
    # a rebuilt lab action); verify() reads every pending flag, any dtype, in one copy
    return DeviceCheck(flag.reshape(-1)[:1], make_exc)


def verify(checks: Iterable[Optional[DeviceCheck]]) -> None:
    """Read every pending flag with ONE device->host copy and raise the first failed check."""
    cs: List[DeviceCheck] = [c for c in checks if c is not None]
    if not cs:
        return
    flags = torch.cat([c.flag for c in cs]).cpu().tolist()  # (cat promotes mixed flag dtypes)
    for c, f in zip(cs, flags):
        if f:
            raise c.make_exc()
