# round-6 GPU call: the library's JIT kernel inside kb3 (same process,
# same placement as the whole-matrix probe), plus the run-time four-Russians prototype
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] kb3"
EC_MI355X_JIT_SYNC=1 timeout -k 10 300 tools/kbench/kb3_r06 1 7 dec16wm > gpurun_out/r06n_kb3_wm.log 2>&1 || { tail -20 gpurun_out/r06n_kb3_wm.log; exit 1; }
cat gpurun_out/r06n_kb3_wm.log
echo "[$(date +%T)] done"
