"""CPU checks of the benchmark entry points: the bench.py JSON contract and the synthetic CSV of
the lab pipeline benchmark (reference data format: CR-only rows, no final terminator)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "benchmarks"))


def test_synth_csv_matches_reference_format(tmp_path):
    import bench_csv_pipeline as B

    p = tmp_path / "s.csv"
    B.synth_csv(str(p), 5000)
    data = p.read_bytes()
    assert b"\n" not in data and data[-1:] != b"\r" and data.count(b"\r") == 4999
    rows = [r.split(b",") for r in data.split(b"\r")]
    g = [int(r[0]) for r in rows]
    pr = [float(r[1]) for r in rows]
    assert min(g) >= 1 and max(g) <= 35 and all(1.0 <= x <= 999.99 for x in pr)
    assert all(len(r[1].split(b".")[1]) in (1, 2) for r in rows)
    assert sum(x < 20 for x in pr) > 0 and sum(a < 14 and x > 90 for a, x in zip(g, pr)) > 0


def test_csv_pipeline_bench_on_host_engine(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "bench_csv_pipeline.py"), "--rows", "20000",
                          "--steps", "1", "--warmup", "0"], capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["unit"] == "rows/s" and line["value"] > 0
    assert 0 < line["config"]["rows_after_dq"] < 20000
    assert abs(line["config"]["coefficients"][0] - 5.0) < 0.3


def test_bench_py_json_contract():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                          "--rows", "50000"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["warmup"] == 1 and line["higher_is_better"] is True
    assert line["metric"].startswith("rows/sec LinearRegression.fit")
    assert line["config"]["coef_max_abs_err"] < 0.05


def test_bench_py_self_launches_ranks():
    """``bench.py --gpus 2`` with no launcher spawns its own two ranks (gloo on this CPU box) and
    reports the two-rank run: n_gpus 2, dp2, one device per rank."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                          "--warmup", "1", "--rows", "40000"], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["backend"] == "gloo" and len(line["rank_devices"]) == 2
    assert line["config"]["coef_max_abs_err"] < 0.05


def test_bench_py_rejects_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="3")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                          "--warmup", "0", "--rows", "1000"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 2 and "WORLD_SIZE=3" in out.stderr


def test_bench_py_under_the_drivers_launcher_four_ranks():
    """The driver's exact multi-GPU command shape (``torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1``), rehearsed with 4 gloo ranks on this CPU box:
    one JSON line from rank 0, strong scaling (global rows fixed, an uneven last shard)."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                          "--gpus", "4", "--steps", "2", "--warmup", "1", "--rows", "40002"],
                         capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 4 and line["world"] == 4 and line["config"]["parallelism"] == "dp4"
    assert line["scaling"] == "strong" and line["config"]["global_batch"] == 40002
    assert line["config"]["coef_max_abs_err"] < 0.05


def _launcher_run(script, args, nproc=4, timeout=900):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, script),
                          "--gpus", str(nproc), *args], capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("script,args", [
    ("benchmarks/bench_dq_pipeline.py", ["--rows-per-gpu", "20000", "--features", "16", "--steps", "1", "--warmup", "1"]),
    ("benchmarks/bench_csv_pipeline.py", ["--rows", "40000", "--steps", "1", "--warmup", "1"]),
    ("benchmarks/bench_wide.py", ["--steps", "1", "--warmup", "1"]),
    ("benchmarks/bench_lbfgs.py", ["--features", "4100", "--rows", "4000", "--max-iter", "15", "--steps", "1",
                                   "--warmup", "0"]),
])
def test_config_benches_under_the_drivers_launcher_four_ranks(script, args, tmp_path, monkeypatch):
    """every config benchmark honours ``--gpus N`` under the driver's launcher shape
    (4 gloo ranks on this CPU box): one JSON line, n_gpus / world 4, one device per rank."""
    monkeypatch.setenv("TMPDIR", str(tmp_path))  # the CSV bench synthesizes its file there
    line = _launcher_run(script, args)
    assert line["n_gpus"] == 4 and line["world"] == 4 and line["backend"] == "gloo"
    assert len(line["rank_devices"]) == 4 and line["config"]["parallelism"] == "dp4"


def test_config_bench_self_launches_and_rejects_mismatch():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "bench_wide.py"), "--gpus", "2",
                          "--steps", "1", "--warmup", "0"], capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["n_gpus"] == 2
    bad = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "bench_dq_pipeline.py"), "--gpus", "2",
                          "--steps", "1", "--warmup", "0"], capture_output=True, text=True, timeout=300,
                         env=dict(env, WORLD_SIZE="3"))
    assert bad.returncode == 2 and "WORLD_SIZE=3" in bad.stderr


def test_scale_curve_script_runs_the_launcher_per_n(tmp_path):
    """scripts/scale_curve.py (the 1/2/4/8 curve in one invocation) on gloo ranks: one record per
    N with the benchmark's own JSON line, and the efficiency table."""
    out = tmp_path / "scale.jsonl"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "scale_curve.py"), "--gpus", "1,2",
                        "--configs", "headline", "--quick", "--out", str(out), "--port", "29871"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    recs = [json.loads(x) for x in out.read_text().splitlines()]
    assert [r["n"] for r in recs] == [1, 2]
    assert all(r["result"]["n_gpus"] == r["n"] for r in recs)
    assert "| headline | 2 |" in p.stdout
