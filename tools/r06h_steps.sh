# round-6 GPU call: the JIT kernel with 4- and 8-stripe tiles: parity, then
# bench.py --only JIT off / T4 / T8 alternating
set -u
mkdir -p gpurun_out
for t in 4 8; do
  echo "[$(date +%T)] pytest jit T=$t"
  EC_MI355X_JIT_T=$t timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06h_pytest_jit_t$t.log 2>&1 || { tail -40 gpurun_out/r06h_pytest_jit_t$t.log; exit 1; }
  tail -2 gpurun_out/r06h_pytest_jit_t$t.log
done
echo "[$(date +%T)] bench"
for r in 1 2 3; do
  for v in "0 4" "1 4" "1 8"; do
    set -- $v
    for cfg in dec:16+4:FFFF0 dec:16+4:F0FFF; do
      out=$(EC_MI355X_JIT=$1 EC_MI355X_JIT_T=$2 EC_MI355X_JIT_SYNC=1 EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only $cfg --gib 1 --steps 40 --warmup 10 --warm-ms 150 2>/dev/null | grep '^{') || exit 1
      echo "{\"round\": $r, \"jit\": $1, \"T\": $2, \"res\": $out}"
    done
  done
done > gpurun_out/r06h_jitab.log 2>&1
cat gpurun_out/r06h_jitab.log
echo "[$(date +%T)] done"
