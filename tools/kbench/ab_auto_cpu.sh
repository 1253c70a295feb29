#!/bin/bash
# Alternating same-box A/B of the CPU path cost of host calls: the CPU
# engine alone (cpu-extensions=avx), auto (GPU engine loaded, the call routed
# to the CPU by the cost model), and auto with EC_CPU_BELOW_KB forcing the
# CPU before the cost model runs.
set -u
OUT=gpurun_out/${1:-ab_auto_cpu}.log
: > "$OUT"
for cell in "4 1 128 16" "8 1 128 16" "4 0 128 16"; do
  set -- $cell
  for rep in 1 2; do
    for mode in avx auto below; do
      case $mode in avx) G=avx; B=0 ;; auto) G=auto; B=0 ;; below) G=auto; B=100000 ;; esac
      printf "%-6s " $mode >> "$OUT"
      EC_CPU_BELOW_KB=$B EC_MI355X_QUIET=1 timeout -k 10 60 tools/kbench/smallcalls 0.7 $1 $2 0 $3 $4 $G 2>&1 | grep "thr:" >> "$OUT" || exit 1
    done
  done
done
cat "$OUT"
