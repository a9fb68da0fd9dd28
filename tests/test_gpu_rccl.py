"""RCCL (``torch.distributed`` backend ``nccl`` on ROCm) exercised on the one-GPU test box:
``DQ4ML_FORCE_COLLECTIVES=1`` makes a one-rank communicator issue every collective the engine
uses at N GPUs, so the nccl init, the bucketed side-stream all-reduce, the
async health check and the overlapped fit tail are covered before any 8-GPU run."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
_DIST_ENV = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")


def _env():
    env = {k: v for k, v in os.environ.items() if k not in _DIST_ENV}
    env.update(DQ4ML_FORCE_COLLECTIVES="1", DQ4ML_COMM_TIMEOUT="60", HSA_ENABLE_IPC_MODE_LEGACY="0")
    return env


@pytest.fixture(scope="module")
def rccl_run():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = subprocess.run([sys.executable, os.path.join(HERE, "_gpu_rccl_worker.py")], env=_env(),
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_rccl_backend_initialised(rccl_run):
    assert rccl_run["backend"] == "nccl" and rccl_run["world"] == 1 and rccl_run["active"]
    assert rccl_run["rccl_version"]


def test_rccl_comm_entry_points(rccl_run):
    for k in ("sum_small", "sum_host", "sum_bucketed", "max", "broadcast", "gather_obj", "health"):
        assert rccl_run[k] is True, k


def test_rccl_fit_paths_match_uncollective(rccl_run):
    assert rccl_run["fit_sync_eq"] and rccl_run["fit_async_eq"] and rccl_run["wide_eq"]
    assert rccl_run["async_in_flight"] and rccl_run["async_many"]
    assert rccl_run["coef_err"] < 5e-3


def test_rccl_lbfgs_per_evaluation_all_reduce(rccl_run):
    """K9 + X4: the squared-loss l-bfgs path all-reduces its (d + 1)-f64 evaluation once per cost
    evaluation over RCCL and ends with the same model as the collective-free run."""
    assert rccl_run["lbfgs_eq"]
    assert rccl_run["lbfgs_allreduce_calls"] >= 5


def test_rccl_wide_banded_fold_all_reduce(rccl_run):
    """Wide Gram X1: band-by-band fold with each band's all-reduce in flight during the next fold."""
    assert rccl_run["wide_bands"] >= 3
    assert rccl_run["wide_banded_f64_eq"]
    assert rccl_run["wide_banded_f32_diff"] < 1e-4
    # the head band stays f64 on the wire (a count above 2^24 is exact)
    assert rccl_run["head_band_count_exact"]


def test_rccl_calls_observed(rccl_run):
    """Only RCCL all-reduces are inside the profiled region.  A one-rank in-place all-reduce is
    a no-op on the device (RCCL's one-rank path launches no ring kernel), so what is visible is
    ProcessGroupNCCL's stream ordering around each call: an event on the caller's stream that
    the communicator stream waits on.  With N ranks the same calls launch ``ncclDevKernel_*``."""
    if not rccl_run["kernels"]:
        pytest.skip("torch profiler saw no HIP activity on this box: " + rccl_run.get("profiler_error", ""))
    names = set(rccl_run["kernels"])
    assert rccl_run["rccl_kernel_seen"] or {"hipEventRecord", "hipStreamWaitEvent"} <= names, names


def test_bench_py_over_rccl():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--rows", "2e6"], env=_env(), capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["backend"] == "nccl" and line["n_gpus"] == 1 and line["rccl_version"]
    assert line["config"]["coef_max_abs_err"] < 5e-3
