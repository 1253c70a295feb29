#!/bin/bash
# Validation at HEAD on the GPU box: smoke -> gpu tests -> bench.
# Stops at the first crash/abort/timeout (no retries).
set -u
mkdir -p gpurun_out
TAG=${TAG:-check}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -4 "gpurun_out/${TAG}_$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run bench 400 python -u bench.py
