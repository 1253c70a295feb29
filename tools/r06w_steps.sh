# round-6 GPU call: 16+4 host-buffer encodes as a combine with the encode
# matrix (r06): the new host-path tests and the knob test, then pinned 16+4
# encode / decode / heal by size, EC_MI355X_ZCENC16=0 (register encoder)
# against the default, alternating, 2 rounds
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] pytest"
timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread -m gpu \
  tests/test_gpu_host_paths.py tests/test_gpu_knobs.py > gpurun_out/r06w_pytest.log 2>&1 || { tail -30 gpurun_out/r06w_pytest.log; exit 1; }
tail -3 gpurun_out/r06w_pytest.log
echo "[$(date +%T)] zc_sizes"
for r in 1 2; do for v in 0 1; do
  EC_GPU_ALWAYS=1 EC_MI355X_ZCENC16=$v ZC_GEOS="16+4" ZC_SIZES="16 64 256 512" timeout -k 10 300 python3 tools/zc_sizes.py >> gpurun_out/r06w_zcsizes.log 2>&1 || { tail -20 gpurun_out/r06w_zcsizes.log; exit 1; }
done; done
cat gpurun_out/r06w_zcsizes.log
echo "[$(date +%T)] done"
