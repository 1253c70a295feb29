#!/bin/bash
# Sustained A/B of the output tile modes (default EC_MI355X_OT=3 vs 1 on
# k = 8; OTS / CFGS override, e.g. OTS="1 4" CFGS="dec:16+4:FFFF0"): 100
# timed launches after 300 warm-up launches (~0.1 s of continuous load).
set -u
for rep in 1 2 3; do
  for o in ${OTS:-1 3}; do
    for cfg in ${CFGS:-dec:8+4:FF0 mixed:8+4}; do
      printf "OT=%s %s rep%s " "$o" "$cfg" "$rep"
      EC_MI355X_OT=$o EC_MI355X_QUIET=1 timeout -k 10 100 python3 bench.py --only $cfg \
        --steps 100 --warmup 300 2>/dev/null | tail -1 || exit 1
    done
  done
done
