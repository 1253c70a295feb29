#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02g}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -3 "gpurun_out/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
run bench 700 python -u bench.py
run xover 400 bash tools/kbench/xover_cells.sh ${TAG}_xover_cells
run profile 900 bash tools/profile.sh $TAG dec:4+2:3C 1 enc:4+2 1 dec:8+4:FF0 0.25 enc:8+4 0.25 dec:16+4:FFFF0 1 enc:16+4 2 mixed:8+4 1 mixed:8+4:16:1 1 heal:8+4 1
