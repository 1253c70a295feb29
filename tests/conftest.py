import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE sizes)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # test infrastructure only
    O.lib()
    return O


# The GPU tests compare the gfx950 kernels with the oracle, so host-buffer
# calls must reach the GPU whatever their size: switch the CPU/GPU crossover
# off for this process (read once, when the library first codes).  The
# crossover itself is tested in a child process with the defaults
# (tests/test_gpu_engine.py).
os.environ.setdefault("EC_GPU_ALWAYS", "1")
