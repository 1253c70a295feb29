# round-6 GPU call: JIT on / off through bench.py --only after the warm-up
# fix (first call outside the warm-up clock), 16+4 decodes and 12+4-class
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] bench"
for r in 1 2 3; do
  for v in 0 1; do
    for cfg in dec:16+4:FFFF0 dec:16+4:F0FFF dec:16+4:5FFF5; do
      out=$(EC_MI355X_JIT=$v EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only $cfg --gib 1 --steps 40 --warmup 10 --warm-ms 150 2>/dev/null | grep '^{') || exit 1
      echo "{\"round\": $r, \"jit\": $v, \"res\": $out}"
    done
  done
done > gpurun_out/r06j_jitab.log 2>&1
cat gpurun_out/r06j_jitab.log
echo "[$(date +%T)] done"
