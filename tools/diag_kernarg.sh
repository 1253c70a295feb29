#!/bin/bash
# Same kernels, two HIP runtimes: kb3 (linked against /opt/rocm 7.2) and the
# library under torch's bundled runtime (bench.py --only), with the kernel
# arguments forced to device memory or not.  Output: gpurun_out/kernarg_*.log
set -u
mkdir -p gpurun_out
O=gpurun_out/kernarg_summary.log
: > $O
for cfg in dec:4+2:3C dec:8+4:FF0 dec:16+4:FFFF0 mixed:16+4:64; do
  for kv in default 1 0; do
    if [ $kv = default ]; then
      timeout -k 10 120 python -u bench.py --only $cfg --gib 1 --steps 100 --warmup 20 > gpurun_out/kernarg_run.log 2>&1 || exit $?
    else
      HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 120 python -u bench.py --only $cfg --gib 1 --steps 100 --warmup 20 > gpurun_out/kernarg_run.log 2>&1 || exit $?
    fi
    echo "$cfg HIP_FORCE_DEV_KERNARG=$kv $(grep '^{' gpurun_out/kernarg_run.log)" >> $O
  done
done
timeout -k 10 300 tools/kbench/kb3 1 7 dec4,dec8,dec16,mixed16 > gpurun_out/kernarg_kb3.log 2>&1 || exit $?
cat $O
