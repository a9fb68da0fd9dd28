"""``master`` chooses the parallel width — ``mi355x[N]`` = N ranks (one process per
GPU), ``local[N]`` = N threads; inside a launcher the group must match, outside one an explicit
SPMD width starts its own ranks."""
import json
import os
import subprocess
import sys

import pytest

from net.jgp.labs.sparkdq4ml_amd.sql.session import master_width

HERE = os.path.dirname(os.path.abspath(__file__))
_DIST_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")


def test_master_width_parse():
    assert master_width("mi355x[4]", "cuda") == 4
    assert master_width("local[2]", "cpu") == 2
    assert master_width("local[3, 2]", "cpu") == 3  # local[N, maxFailures]
    assert master_width("local", "cpu") == 1
    assert master_width("local[*]", "cpu") == (os.cpu_count() or 1)
    with pytest.raises(ValueError):
        master_width("local[0]", "cpu")


def test_explicit_spmd_width_starts_its_ranks():
    env = {k: v for k, v in os.environ.items() if k not in _DIST_ENV}
    env["DQ4ML_DEVICE"] = "cpu"
    p = subprocess.run([sys.executable, os.path.join(HERE, "_master_width_worker.py")], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = sorted((json.loads(x) for x in p.stdout.strip().splitlines() if x.startswith("{")), key=lambda r: r["rank"])
    assert [r["rank"] for r in lines] == [0, 1]
    assert all(r["world"] == 2 and r["width"] == 2 for r in lines)
    assert [r["count"] for r in lines] == [20, 20]  # range() is per-rank data; count() is global


def test_width_mismatch_inside_a_group(monkeypatch):
    from net.jgp.labs.sparkdq4ml_amd.sql import session as S

    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(ValueError, match="process group has 2"):
        S._launch_width("mi355x[3]", 3, True)
