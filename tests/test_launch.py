"""The one-process-per-GPU launcher: env wiring, data-parallel run, fail-fast on a dead rank."""
import sys
import textwrap

from net.jgp.labs.sparkdq4ml_amd.parallel.launch import launch


def _script(tmp_path, body):
    p = tmp_path / "w.py"
    p.write_text(textwrap.dedent(body))
    return str(p)


def test_launch_runs_a_gloo_group(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    s = _script(tmp_path, f"""
        import os, sys
        sys.path.insert(0, {repr(str(__import__('os').path.dirname(__import__('os').path.dirname(__file__))))})
        os.environ["DQ4ML_DEVICE"] = "cpu"
        import torch
        from net.jgp.labs.sparkdq4ml_amd.parallel import comm
        comm.init(backend="gloo")
        t = comm.all_reduce_sum(torch.tensor([float(comm.rank() + 1)]))
        open(os.path.join({repr(str(out))}, str(comm.rank())), "w").write(str(float(t[0])))
        comm.shutdown()
    """)
    assert launch(3, [s]) == 0
    assert sorted(p.name for p in out.iterdir()) == ["0", "1", "2"]
    assert all(p.read_text() == "6.0" for p in out.iterdir())


def test_launch_fails_fast(tmp_path):
    s = _script(tmp_path, """
        import os, sys, time
        if os.environ["RANK"] == "1":
            sys.exit(3)
        time.sleep(60)  # would hang without fail-fast
    """)
    import time

    t0 = time.time()
    assert launch(3, [s], grace_s=2.0) == 3
    assert time.time() - t0 < 30
