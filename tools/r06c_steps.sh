# round-6 GPU call: the whole-matrix k = 16 probe, then the GPU suite, smoke and bench
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] kb3 dec16wm"
timeout -k 10 300 tools/kbench/kb3_r06 1 7 dec16wm > gpurun_out/r06c_kb3_wm.log 2>&1; rc=$?
cat gpurun_out/r06c_kb3_wm.log | tail -15
[ $rc -eq 0 ] || exit $rc
TAG=r06c bash tools/gpu_steps.sh smoke pytest bench
