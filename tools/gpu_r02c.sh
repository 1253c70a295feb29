#!/bin/bash
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02c}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -4 "gpurun_out/${TAG}_$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run kbench 400 env KB_NO_ENCODE=1 tools/kbench/kbench 1 7
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
run bench_2rank 600 env EC_BENCH_BACKEND=gloo EC_BENCH_DEVICE=0 python -u bench.py --gpus 2 --steps 5 --warmup 1
run bench 600 python -u bench.py
run pmc16 400 bash tools/pmc_r02.sh dec16p4 dec:16+4:FFFF0 1
