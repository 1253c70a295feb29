# round-6 GPU call: the 64-mask 16+4 mixed call, library path vs the device-table kernel with its table resident
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] kb3"
timeout -k 10 400 tools/kbench/kb3_r06 1 7 mixed16s > gpurun_out/r06q_kb3_mixed.log 2>&1 || { tail -20 gpurun_out/r06q_kb3_mixed.log; exit 1; }
cat gpurun_out/r06q_kb3_mixed.log
echo "[$(date +%T)] done"
