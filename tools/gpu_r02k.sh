#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02k}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -3 "gpurun_out/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run kbench 400 env KB_NO_ENCODE=1 tools/kbench/kbench 1 7
run pytest_engine 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v --timeout 200 --timeout-method thread
run xover 500 env SECS=0.7 bash tools/kbench/xover_cells.sh ${TAG}_xover_pageable
run xover_reg 500 env SECS=0.7 REG=1 bash tools/kbench/xover_cells.sh ${TAG}_xover_registered
du -sh gpurun_out
