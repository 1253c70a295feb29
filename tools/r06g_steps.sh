# round-6 GPU call: placement of the fragments and the JIT kernel (kb3,
# contiguous vs separate allocations), then bench.py JIT on/off by placement
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] kb3"
EC_MI355X_JIT_SYNC=1 timeout -k 10 300 tools/kbench/kb3_r06 1 7 dec16wm > gpurun_out/r06g_kb3_wm.log 2>&1 || { tail -20 gpurun_out/r06g_kb3_wm.log; exit 1; }
cat gpurun_out/r06g_kb3_wm.log
echo "[$(date +%T)] bench placement x jit"
for r in 1 2; do
  for st in 0 4096 262144; do
    for v in 0 1; do
      out=$(EC_BENCH_FRAG_STAGGER=$st EC_MI355X_JIT=$v EC_MI355X_JIT_SYNC=1 EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only dec:16+4:FFFF0 --gib 1 --steps 40 --warmup 10 --warm-ms 150 2>/dev/null | grep '^{') || exit 1
      echo "{\"round\": $r, \"stagger\": $st, \"jit\": $v, \"res\": $out}"
    done
  done
done > gpurun_out/r06g_placejit.log 2>&1
cat gpurun_out/r06g_placejit.log
echo "[$(date +%T)] done"
echo "[$(date +%T)] concur: 128 KiB writes alone, auto / cpu alternating"
for r in 1 2 3 4; do
  for m in auto avx; do
    EC_GPU_ALWAYS=0 EC_MI355X_QUIET=1 CONCUR_SCEN=write CONCUR_WAYS=concurrent timeout -k 10 60 tools/kbench/concur 1 $m pool 2>/dev/null || exit 1
  done
done > gpurun_out/r06g_concur_write.log 2>&1
cat gpurun_out/r06g_concur_write.log
echo "[$(date +%T)] done"
