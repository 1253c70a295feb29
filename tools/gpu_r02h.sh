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
run bench_rocprof 600 bash -c 'cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench_r02h -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-extra --no-cpu && python3 $GRAFT_REPO_ROOT/tools/prof_filter.py $GRAFT_REPO_ROOT/gpurun_out/prof_bench_r02h ecdev'
du -sh gpurun_out
