"""The multi-rank bench path on the GPU: two ranks
started the way the driver starts N > 1 (torch.distributed.run, one process
per rank), both pinned to GPU 0 with the gloo backend because this box has
one GPU (RCCL needs a device per rank).  Each rank decodes its own stripe
range of the one xorshift stream; the control-plane collectives (barrier,
max of the elapsed time, the parity flag, the placement report) must agree,
and rank 0's input, fragments and output must match the oracle's full-size
SHA-256 fixture for its slice."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_two_ranks_on_one_gpu():
    env = dict(os.environ, EC_BENCH_BACKEND="gloo", EC_BENCH_DEVICE="0", EC_MI355X_QUIET="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.pop("EC_GPU_ALWAYS", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--no-extra", "--no-cpu"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "weak"
    assert d["parity_ok"] is True and d["fullsize_sha256_check"] is True
    assert d["config"]["stripes_per_gpu"] == 524288
    assert len(d["ranks"]) == 2 and all(rk["device"] == 0 for rk in d["ranks"])
    assert d["value"] > 0 and d["roofline"]["avg_launch_ms"] > 0
