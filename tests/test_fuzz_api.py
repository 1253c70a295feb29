"""Short runs of the differential fuzzer (tools/fuzz_api.py): random
concurrent calls of every host entry point (encode, row-masked encode,
decode, mixed decode, heal, partial write, the reference's size-based pair)
over eleven geometries and every buffer kind, each compared byte for byte
with the oracle.  The CPU-suite run codes on the library's CPU engine (no
device here); the GPU run keeps every host call on the GPU (EC_GPU_ALWAYS=1)
and adds device, odd-offset device and registered buffers.  A fixed seed
makes a failure replayable (FUZZ_SEED)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "fuzz_api.py")


def _run(secs, seed, extra_env):
    env = dict(os.environ, FUZZ_SECS=str(secs), FUZZ_THREADS="4", FUZZ_SEED=str(seed),
               EC_MI355X_QUIET="1", **extra_env)
    r = subprocess.run([sys.executable, TOOL], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=secs + 120)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, (r.stdout[-2000:], r.stderr[-2000:])
    res = json.loads(lines[-1])
    assert not res["mismatches"] and sum(res["calls"].values()) > 0, res
    return res


def test_fuzz_cpu_engine():
    import glusterfs_amd as g
    if g.device_count() > 0:
        pytest.skip("GPU visible: the GPU variant covers this")
    res = _run(6, 4242, {})
    assert res["cpu_calls"] > 0


@pytest.mark.gpu
def test_fuzz_gpu_always():
    res = _run(25, 4243, {"EC_GPU_ALWAYS": "1"})
    assert res["gpu_calls"] > 0 and res["cpu_fallbacks"] == 0
