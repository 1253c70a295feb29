# Development probe: a subset of tools/kbench/smallcalls cells (op, buffers,
# size, threads) plus the 512 MiB host-buffer rates of tools/kbench/e2e.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/${1:-sc_cells}.log
: > $OUT
for k in 4 8; do
  for dec in 0 1; do
    for reg in 1 0; do
      for kib in 128 1024 4096; do
        for thr in 1 16; do
          timeout -k 10 60 tools/kbench/smallcalls ${SECS:-0.4} $k $dec $reg $kib $thr 2>/dev/null | grep thr: >> $OUT || exit 1
        done
      done
    done
  done
done
timeout -k 10 200 tools/kbench/e2e 512 3 >> $OUT 2>&1 || exit 1
