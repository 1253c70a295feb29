# round-6 GPU call: JIT parity, then kb3's whole-matrix probe and the
# library's JIT on / off through bench.py --only on the same box
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] pytest jit"
timeout -k 10 600 python -u -m pytest tests/test_gpu_jit.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06e_pytest_jit.log 2>&1 || { tail -40 gpurun_out/r06e_pytest_jit.log; exit 1; }
tail -3 gpurun_out/r06e_pytest_jit.log
echo "[$(date +%T)] kb3"
timeout -k 10 300 tools/kbench/kb3_r06 1 5 dec16wm > gpurun_out/r06e_kb3_wm.log 2>&1 || exit 1
tail -10 gpurun_out/r06e_kb3_wm.log
echo "[$(date +%T)] jit ab"
for r in 1 2 3; do
  for v in 0 1; do
    for cfg in dec:16+4:FFFF0 dec:16+4:F0FFF; do
      out=$(EC_MI355X_JIT=$v EC_MI355X_JIT_SYNC=1 EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only $cfg --gib 1 --steps 40 --warmup 10 --warm-ms 150 2>/dev/null | grep '^{') || exit 1
      echo "{\"round\": $r, \"jit\": $v, \"res\": $out}"
    done
  done
done > gpurun_out/r06e_jitab.log 2>&1
cat gpurun_out/r06e_jitab.log
echo "[$(date +%T)] done"
