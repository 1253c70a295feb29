# round-6 GPU call: the device-table (PG) kernels reading their pattern by
# scalar loads (no LDS copy): mixed-pattern parity tests, then kb3's mixed
# groups (device-table kernel against the argument-space one, same patterns)
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] pytest mixed"
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_guards.py tests/test_gpu_errors.py tests/test_gpu_host_paths.py \
  tests/test_gpu_concurrency.py tests/test_gpu_fullsize.py -k "mixed or table or heal or fullsize or 16p4" \
  > gpurun_out/r06t_pytest_mixed.log 2>&1 || { tail -30 gpurun_out/r06t_pytest_mixed.log; exit 1; }
tail -3 gpurun_out/r06t_pytest_mixed.log
echo "[$(date +%T)] kb3"
timeout -k 10 400 tools/kbench/kb3_r06 1 7 mixed16s,mixed8s > gpurun_out/r06t_kb3_mixed.log 2>&1 || { tail -20 gpurun_out/r06t_kb3_mixed.log; exit 1; }
cat gpurun_out/r06t_kb3_mixed.log
echo "[$(date +%T)] done"
