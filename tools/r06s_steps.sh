# round-6 GPU call: mixed calls after the device-table kernel loads its pattern in wave 0 only
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] kb3"
timeout -k 10 400 tools/kbench/kb3_r06 1 7 mixed16s,mixed8s > gpurun_out/r06s_kb3_mixed.log 2>&1 || { tail -20 gpurun_out/r06s_kb3_mixed.log; exit 1; }
cat gpurun_out/r06s_kb3_mixed.log
echo "[$(date +%T)] done"
