#!/bin/bash
# Same-box A/B of the device pattern-table cache (EC_MI355X_PATCACHE=0 / 1)
# on mixed decodes past the argument space, alternating processes.
set -u
for rep in 1 2 3; do
  for c in 0 1; do
    for cfg in mixed:16+4:64 mixed:8+4:64; do
      printf "PATCACHE=%s %s rep%s " "$c" "$cfg" "$rep"
      EC_MI355X_PATCACHE=$c EC_MI355X_QUIET=1 timeout -k 10 100 python3 bench.py --only $cfg \
        --steps 40 --warmup 20 2>/dev/null | tail -1 || exit 1
    done
  done
done
