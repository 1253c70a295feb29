#!/bin/bash
# Round-end evidence at HEAD: smoke -> gpu tests -> 2-rank rehearsal (gloo,
# both ranks on GPU 0) -> bench -> rocprofv3 trace + PMC passes.
# Stops at the first failure (no retries).
set -u
TAG=${TAG:-final}
bash tools/gpu_check.sh || exit $?
echo "[$(date +%T)] start rehearsal"
timeout -k 10 300 env EC_BENCH_BACKEND=gloo EC_BENCH_DEVICE=0 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 1 > "gpurun_out/${TAG}_rehearsal.log" 2>&1 || exit $?
tail -1 "gpurun_out/${TAG}_rehearsal.log" | cut -c1-300
echo "[$(date +%T)] start profile"
timeout -k 10 900 bash tools/profile.sh "$TAG" dec:4+2:3C 1 enc:4+2 1 enc:8+4 0.25 dec:8+4:FF0 0.25 \
  enc:16+4 2 mixed:8+4 1 heal:8+4 1 dec:16+4:FFFF0 1 mixed:16+4:64 1 rmw:4+2 1 \
  > "gpurun_out/${TAG}_profile.log" 2>&1 || exit $?
echo "[$(date +%T)] done"
