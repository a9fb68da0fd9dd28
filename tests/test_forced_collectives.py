"""``DQ4ML_FORCE_COLLECTIVES=1`` on one CPU process: a one-rank gloo group, every collective
issued (the CPU twin of ``test_gpu_rccl.py``)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CODE = r"""
import json, sys, torch
sys.path.insert(0, %r)
from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession
from net.jgp.labs.sparkdq4ml_amd.parallel import comm
comm.init()
out = {"backend": comm.backend(), "active": comm.collectives_active(), "world": comm.world_size()}
x = torch.arange(5, dtype=torch.float64)
out["sum"] = comm.all_reduce_sum(x.clone()).tolist() == x.tolist()
out["gather"] = comm.all_gather_object(3) == [3]
comm.health_check(10)
spark = SparkSession.builder().master("cpu").getOrCreate()
g = torch.Generator().manual_seed(0)
X = torch.randn(3, 5000, generator=g, dtype=torch.float64)
y = torch.tensor([1.0, -2.0, 0.5], dtype=torch.float64) @ X + 4
m = LinearRegression(solver="normal").fit(spark.createDataFrame({"features": X, "label": y}))
out["coef"] = m.coefficients.toArray().tolist()
out["r2"] = float(m.summary.r2)
comm.shutdown()
print(json.dumps(out))
""" % ROOT


def test_forced_collectives_one_rank_gloo():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["DQ4ML_FORCE_COLLECTIVES"] = "1"
    p = subprocess.run([sys.executable, "-c", _CODE], env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    o = json.loads(p.stdout.strip().splitlines()[-1])
    assert o["backend"] == "gloo" and o["active"] and o["world"] == 1
    assert o["sum"] and o["gather"]
    assert max(abs(a - b) for a, b in zip(o["coef"], [1.0, -2.0, 0.5])) < 1e-9 and o["r2"] > 0.999999
