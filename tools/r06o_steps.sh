# round-6 GPU call: what the mixed-pattern combine costs over the
# single-pattern one (kb3 mixed8 / mixed16 with two controls: the mixed map
# with every group on pattern 0, and pattern 0 as a plain call), plus dec8
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] kb3"
timeout -k 10 300 tools/kbench/kb3_r06 1 7 mixed8,mixed16,dec8 > gpurun_out/r06o_kb3_mixed.log 2>&1 || { tail -20 gpurun_out/r06o_kb3_mixed.log; exit 1; }
cat gpurun_out/r06o_kb3_mixed.log
echo "[$(date +%T)] done"
