#!/bin/bash
# Alternating same-box A/B of the CPU path cost: cpu-extensions=avx in a
# process without HIP, the same with the gfx950 engine initialised beside it
# (SC_PREINIT=1), and auto (GPU engine, calls routed to the CPU).
set -u
OUT=gpurun_out/${1:-ab_auto_cpu}.log
: > "$OUT"
for cell in "4 0 128 16" "4 1 1024 16" "4 1 1024 1"; do
  set -- $cell
  for rep in 1; do
    for mode in avx avxpre auto; do
      case $mode in avx) G=avx; P=0 ;; avxpre) G=avx; P=1 ;; auto) G=auto; P=0 ;; esac
      printf "%-6s " $mode >> "$OUT"
      EC_MI355X_DEBUG=1 SC_PREINIT=$P EC_MI355X_QUIET=1 timeout -k 10 60 tools/kbench/smallcalls 0.7 $1 $2 0 $3 $4 $G 2>&1 | grep "thr:\|queries" | tr '\n' ' ' >> "$OUT" || exit 1
      echo >> "$OUT"
    done
  done
done
cat "$OUT"
