# round-6 GPU call: mixed-pattern combines with disjoint fragments (as the
# dense decode groups), incl. the bench's 64-mask 16+4 call through the
# library's device-table path, beside the single-pattern controls
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] kb3"
timeout -k 10 400 tools/kbench/kb3_r06 1 7 mixed8s,mixed16s,dec8 > gpurun_out/r06p_kb3_mixed.log 2>&1 || { tail -20 gpurun_out/r06p_kb3_mixed.log; exit 1; }
cat gpurun_out/r06p_kb3_mixed.log
echo "[$(date +%T)] done"
