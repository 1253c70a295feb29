#!/bin/bash
# Same-box A/B of the device encoders under sustained load: alternating
# processes, EC_MI355X_ENC=0 (register-resident) / 1 (tile kernels), 60
# timed launches after 20 warmup launches each.
set -u
OUT=gpurun_out/${1:-ab_enc}.log
: > "$OUT"
for cfg in enc:4+2 enc:8+4 enc:16+4; do
  for rep in 1 2; do
    for e in 0 1; do
      echo -n "ENC=$e $cfg rep$rep " >> "$OUT"
      EC_MI355X_ENC=$e EC_MI355X_QUIET=1 timeout -k 10 200 python3 bench.py --only $cfg --steps 60 --warmup 20 2>/dev/null | tail -1 >> "$OUT" || exit 1
    done
  done
done
cat "$OUT"
