#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02h}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -3 "gpurun_out/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
run xover 400 bash tools/kbench/xover_cells.sh ${TAG}_xover_pageable
run xover_reg 400 env REG=1 bash tools/kbench/xover_cells.sh ${TAG}_xover_registered
run e2e 400 bash tools/kbench/e2e_sweep.sh ${TAG}_e2e
du -sh gpurun_out
