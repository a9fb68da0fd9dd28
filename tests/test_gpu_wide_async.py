"""The asynchronous wide normal-equation fit (BASELINE config 5's path): enqueued end to end with
no host sync (``sync_debug_mode("error")``), one-rank forced RCCL and without collectives, and
bit-identical to the synchronous fit of the same statistics (same PCG iterates: converged
iterations are no-ops)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["local", "rccl"])
@pytest.mark.parametrize("eb", [8, 16])
def test_wide_async_fit_no_host_sync(mode, eb):
    import socket

    here = os.path.dirname(os.path.abspath(__file__))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", DQ4ML_COMM_TIMEOUT="60")
    p = subprocess.run([sys.executable, os.path.join(here, "_gpu_wide_async_worker.py"), mode, str(eb)], env=env,
                       capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stderr[-3000:]
    o = json.loads(p.stdout.strip().splitlines()[-1])
    ref = np.asarray(o["ref_coef"])
    assert o["solver"] == "cholesky"
    for c, icpt in zip(o["coef"], o["icpt"]):
        np.testing.assert_allclose(np.asarray(c), ref, rtol=1e-12, atol=1e-13)
        assert icpt == pytest.approx(o["ref_icpt"], rel=1e-12, abs=1e-13)
    # the model is the regression it should be (fp8 / bf16 features: a few % on coefficients)
    beta = np.linspace(-1.0, 1.0, ref.size)
    assert np.abs(ref - beta).max() < (0.1 if eb == 8 else 0.02)
