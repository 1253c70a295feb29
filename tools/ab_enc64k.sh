#!/bin/bash
# Same-box A/B of the 8+4 encoder on 64K-stripe batches (BASELINE configs[2]):
# register-resident (EC_MI355X_ENC unset) vs tile (=2), alternating
# processes, 200 timed launches after 50 warm-up launches.
set -u
OUT=gpurun_out/${1:-ab_enc64k}.log
: > "$OUT"
for rep in 1 2 3; do
  for e in 1 2; do
    echo -n "ENC=$e enc:8+4 0.25GiB rep$rep " >> "$OUT"
    EC_MI355X_ENC=$e EC_MI355X_QUIET=1 timeout -k 10 200 python3 bench.py --only enc:8+4 --gib 0.25 --steps 200 --warmup 50 2>/dev/null | tail -1 >> "$OUT" || exit 1
  done
done
cat "$OUT"
