"""Rehearse the data-parallel fit with 2 ranks on ONE GPU box: both ranks use cuda:0 for compute
and the gloo backend for the collectives (RCCL needs one GPU per rank).  Checks every rank gets
the single-process model."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["LOCAL_RANK"] = "0"  # both ranks share the only GPU
from net.jgp.labs.sparkdq4ml_amd import LinearRegression, SparkSession  # noqa: E402
from net.jgp.labs.sparkdq4ml_amd.parallel import comm  # noqa: E402

comm.init(backend="gloo")
rank, world = comm.rank(), comm.world_size()
g = torch.Generator(device="cuda").manual_seed(0)
n, d = 2_000_000, 32
X = torch.randn(d, n, generator=g, device="cuda")
y = torch.linspace(-1, 1, d, device="cuda") @ X + 0.5
lo, hi = rank * n // world, (rank + 1) * n // world
spark = SparkSession.builder().master("mi355x[*]").getOrCreate()
df = spark.createDataFrame({"features": X[:, lo:hi].to(torch.bfloat16), "label": y[lo:hi].contiguous()})
m = LinearRegression(solver="normal", gramDtype="bf16").fit(df)
coef = torch.tensor(m.coefficients.toArray())
allc = comm.all_gather_object(coef.tolist())
assert all(c == allc[0] for c in allc), "ranks disagree"
assert m.summary.numInstances == n, m.summary.numInstances
err = float((coef - torch.linspace(-1, 1, d, dtype=torch.float64)).abs().max())
print(f"rank {rank}: numInstances={m.summary.numInstances} max|coef-beta|={err:.3e} r2={m.summary.r2:.6f}")
assert err < 5e-3
# asynchronous fits with the overlapped tail (all-reduce + device solve on the side stream),
# several in flight before the first read: must equal the synchronous model
spark.conf.set("dq4ml.fit.async", "true")
ms = [LinearRegression(solver="normal", gramDtype="bf16").fit(df) for _ in range(4)]
for ma in ms:
    ca = torch.tensor(ma.coefficients.toArray())
    assert torch.allclose(ca, coef, rtol=1e-9, atol=1e-12), (ca - coef).abs().max()
    assert ma.summary.numInstances == n
spark.conf.set("dq4ml.fit.async", "false")
print(f"rank {rank}: async overlapped fits match")
# sharded large-CSV read: each rank reads / pins / caches only its byte range (filecache.shard_range)
import numpy as np  # noqa: E402

path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "dq4ml_rehearsal.csv")
if rank == 0:
    rng = np.random.default_rng(3)
    gg = rng.integers(1, 36, 300_000)
    open(path, "wb").write("\r".join(f"{int(a)},{5 * int(a) + 20}.5" for a in gg).encode())
comm.barrier()
spark.conf.set("dq4ml.csv.deviceThresholdBytes", "0")
t = spark.read().option("inferSchema", "true").csv(path)._table()
rows = comm.all_gather_object(int(t.nrows))
assert sum(rows) == 300_000, rows
print(f"rank {rank}: sharded device CSV rows {rows}")
comm.barrier()
comm.shutdown()
