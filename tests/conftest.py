import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("DQ4ML_LOG_LEVEL", "ERROR")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture
def cpu_session():
    from net.jgp.labs.sparkdq4ml_amd import SparkSession

    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    s = SparkSession.builder().appName("test").master("cpu").getOrCreate()
    yield s
    s.stop()


@pytest.fixture
def gpu_session():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from net.jgp.labs.sparkdq4ml_amd import SparkSession

    s = SparkSession.getActiveSession()
    if s is not None:
        s.stop()
    s = SparkSession.builder().appName("test").master("mi355x[*]").getOrCreate()
    yield s
    s.stop()


def data_path(name):
    return os.path.join(ROOT, "data", name)
