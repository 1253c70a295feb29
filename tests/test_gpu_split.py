"""The library's in-process multi-device split (ec_device.hip partition())
exercised on one GPU: EC_MI355X_TEST_SPLIT=1 lets EC_MI355X_HOST_DEVICES=0,0
name GPU 0 twice, so every host-buffer call is cut into two stripe ranges
coded by two host threads with their own stages and streams.  Runs in one
child process (the device list is read once per process)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_partition_two_way_on_one_gpu():
    env = dict(os.environ, EC_MI355X_HOST_DEVICES="0,0", EC_MI355X_TEST_SPLIT="1",
               EC_SPLIT_MIN_MB="0", EC_MI355X_QUIET="1")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "_split_child.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "SPLIT-OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
