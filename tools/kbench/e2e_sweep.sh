# Development probe: host-buffer encode/decode rates of the library from a
# torch-free C process (tools/kbench/e2e.c), with and without copy threads.
set -u
mkdir -p gpurun_out
for t in 8 16 0; do
  echo "== copy threads $t" >> gpurun_out/e2e.log
  EC_COPY_THREADS=$t timeout -k 10 200 tools/kbench/e2e 512 3 >> gpurun_out/e2e.log 2>&1 || exit 1
done
