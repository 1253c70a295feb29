# round-6 GPU call: JIT parity tests, then JIT on/off and waves-per-EU A/B
# through bench.py --only (alternating processes, 3 rounds)
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] pytest jit"
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06d_pytest_jit.log 2>&1 || { tail -40 gpurun_out/r06d_pytest_jit.log; exit 1; }
tail -5 gpurun_out/r06d_pytest_jit.log
echo "[$(date +%T)] jit ab"
for r in 1 2 3; do
  for v in "0 0" "1 0"; do
    set -- $v
    for cfg in dec:16+4:FFFF0 dec:16+4:F0FFF; do
      out=$(EC_MI355X_JIT=$1 EC_MI355X_JIT_SYNC=1 EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only $cfg --gib 1 --steps 40 --warmup 10 --warm-ms 150 2>/dev/null | grep '^{') || exit 1
      echo "{\"round\": $r, \"jit\": $1, \"wpe\": $2, \"res\": $out}"
    done
  done
done > gpurun_out/r06d_jitab.log 2>&1
cat gpurun_out/r06d_jitab.log
echo "[$(date +%T)] done"
