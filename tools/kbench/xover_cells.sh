#!/bin/bash
# CPU/GPU crossover cells: GlusterFS-sized calls through
# ec_method_encode / ec_method_decode on pageable buffers from 1 and 16
# threads, each cell three ways: GPU only (crossover off), CPU engine only
# (cpu-extensions=avx), and the library's default crossover.
# REG=1: buffers in a registered (pinned, device-mapped) arena instead.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/${1:-xover}.log
SECS=${SECS:-1.0}
: > "$OUT"
for k in ${KS:-4 8 16}; do
  for dec in ${OPS:-0 1}; do
    for kib in 128 1024 4096 16384; do
      for thr in 1 16; do
        for mode in gpu cpu auto; do
          case $mode in
            gpu)  ENV="EC_GPU_ALWAYS=1"; GEN=auto ;;
            cpu)  ENV=""; GEN=avx ;;
            auto) ENV=""; GEN=auto ;;
          esac
          printf "%-4s " $mode >> "$OUT"
          env $ENV EC_MI355X_QUIET=1 timeout -k 10 60 ${SMALLCALLS:-tools/kbench/smallcalls} ${SECS:-0.5} $k $dec ${REG:-0} $kib $thr $GEN \
            2>/dev/null | grep thr: >> "$OUT" || exit 1
        done
      done
    done
  done
done
