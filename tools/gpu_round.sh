#!/bin/bash
# Full GPU session: smoke -> gpu tests -> 2-rank rehearsal (gloo, one GPU)
# -> bench -> rocprofv3 profiles.  Stops at the first crash/abort/timeout.
set -u
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 1200 python -m pytest tests -m gpu -x -q
step bench_2rank_rehearsal 600 env EC_BENCH_BACKEND=gloo EC_BENCH_DEVICE=0 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 1
step bench 900 python bench.py
if [ "${PROFILE:-1}" = 1 ]; then
  step profile 1000 bash tools/profile.sh ${TAG:-r01d} dec:4+2:3C 1 enc:4+2 1 enc:8+4 0.25 \
    dec:8+4:FF0 0.25 enc:16+4 2 mixed:8+4 1 heal:8+4 1 dec:16+4:FFFF0 1
fi
