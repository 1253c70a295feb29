#!/bin/bash
# Round-2 first GPU session: smoke -> VALU probe -> gpu tests -> 2-rank
# self-launched bench rehearsal (gloo, both ranks on GPU 0) -> bench.
# Stops at the first crash/abort/timeout (no retries).
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02b}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -4 "gpurun_out/${TAG}_$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
run kbench 400 tools/kbench/kbench 1 7
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
run bench_2rank 600 env EC_BENCH_BACKEND=gloo EC_BENCH_DEVICE=0 python -u bench.py --gpus 2 --steps 5 --warmup 1
run bench 600 python -u bench.py
