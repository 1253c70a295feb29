#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02i}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -3 "gpurun_out/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
run kbench 400 env KB_NO_ENCODE=1 tools/kbench/kbench 1 7
run xover 500 bash tools/kbench/xover_cells.sh ${TAG}_xover_pageable
run xover_reg 500 env REG=1 bash tools/kbench/xover_cells.sh ${TAG}_xover_registered
run bench 700 python -u bench.py
du -sh gpurun_out
