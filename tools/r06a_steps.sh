set -o pipefail
mkdir -p gpurun_out
echo "[$(date +%T)] probe"
EC_MI355X_LIB=$PWD/ab_libs/pre.so timeout -k 10 120 python3 bench.py --only rmw:4+2 --gib 1 --steps 10 --warmup 5 > gpurun_out/r06a_probe.log 2>&1 || { tail -30 gpurun_out/r06a_probe.log; exit 1; }
tail -3 gpurun_out/r06a_probe.log
echo "[$(date +%T)] ablib"
AB_LIBS="pre=ab_libs/pre.so head=ab_libs/head.so fix=" ROUNDS=3 timeout -k 10 900 bash tools/ab_lib.sh 'rmw:4+2 1 rmw:8+4 1 rmw:16+4 1 enc:4+2 1 enc:16+4 2' > gpurun_out/r06a_ablib.log 2>&1 || exit 1
echo "[$(date +%T)] pytest"
timeout -k 10 900 python -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_writev.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a_pytest.log 2>&1 || exit 1
echo "[$(date +%T)] done"
