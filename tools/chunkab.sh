# Chunked launches of large single-pattern device calls (EC_MI355X_CHUNK_MB,
# ec_kernels.hip launch_chunk_bytes): parity with 1 MiB launches, then an
# A/B of the chunk size through bench.py --only, after 150 ms of load.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r05ap}
{
timeout -k 10 300 python -u -m pytest tests/test_gpu_knobs.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
for r in 1 2 3; do
 for c in ${CHUNK_CASES:-"enc:16+4 2" "enc:16+4 8" "dec:4+2:3C 2" "enc:8+4 2"}; do
  set -- $c
  for ch in ${CHUNKS:-0 512 1024}; do
   echo "== round $r $1 $2 GiB chunk $ch"
   timeout -k 10 120 env EC_MI355X_CHUNK_MB=$ch python3 bench.py --only $1 --gib $2 --steps 20 --warmup 5 --warm-ms 150 || exit 1
  done
 done
done
} > gpurun_out/${TAG}_chunkab.log 2>&1
