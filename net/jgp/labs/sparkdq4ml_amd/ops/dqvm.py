"""Fused DQ virtual machine (device path).  Filled in with the HIP VM kernel."""
from __future__ import annotations


def try_execute_fused(plan, session):
    return None
