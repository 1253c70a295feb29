#!/bin/bash
# A/B of the LDS-DMA cache policy (default vs non-temporal) on the shipped
# kernels: tools/kbench/kb3 (EC_LDSDMA_AUX=0) and kb3_nt (=2), alternating
# processes.  Output gpurun_out/ab_ldsdma_nt.log
set -u
mkdir -p gpurun_out
O=gpurun_out/ab_ldsdma_nt.log
: > $O
for rd in 1 2 3; do
  for b in kb3 kb3_nt; do
    echo "=== round $rd $b" >> $O
    timeout -k 10 300 tools/kbench/$b 1 5 dec4,dec8,dec16,enc4,enc8,enc16rb > gpurun_out/ab_tmp.log 2>&1 || exit $?
    grep -A1 "^== \|^variant" gpurun_out/ab_tmp.log | grep -v "^--" | grep -v "^variant" >> $O
    grep "^shipped" gpurun_out/ab_tmp.log >> $O
  done
done
cat $O
