# Development probe: host-buffer encode/decode rates of the library from a
# torch-free C process (tools/kbench/e2e.c), over the number of staging copy
# threads (EC_COPY_THREADS; 0 = the calling thread copies alone).
set -u
mkdir -p gpurun_out
OUT=gpurun_out/${1:-e2e}.log
: > "$OUT"
for t in 0 2 8 16; do
  echo "== copy threads $t" >> "$OUT"
  EC_COPY_THREADS=$t EC_MI355X_QUIET=1 timeout -k 10 200 tools/kbench/e2e 512 3 >> "$OUT" 2>&1 || exit 1
done
