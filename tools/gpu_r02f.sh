#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02f}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -3 "gpurun_out/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
run small_groups 300 bash -c 'for c in mixed:8+4:16:1 mixed:8+4:16:2 mixed:8+4:16:4 mixed:8+4:16:8 mixed:16+4:16:1 mixed:16+4:16:8 mixed:4+2:15:1 mixed:4+2:15:8; do printf "%s " $c; EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only $c --gib 1 --steps 10 --warmup 2 || exit 1; done'
run ab_jt 500 bash tools/ab_jt.sh 2 mixed:8+4 1 dec:8+4:FF0 1 dec:8+4:FF0 0.25 mixed:16+4:64 1 dec:4+2:3C 1
run bench 700 python -u bench.py
