#!/bin/bash
# Same-box A/B of the waves per block of the k <= 8 combine kernels through
# the product launcher (EC_MI355X_NW8, or $KNOB, e.g. EC_MI355X_NW4),
# alternating processes, 40 timed launches after 20 warm-up launches.
# Usage: [KNOB=EC_MI355X_NW4] tools/ab_nw8.sh ROUNDS "NW..." CONFIG GIB [...]
set -u
ROUNDS=$1; NWS=$2; shift 2
while [ $# -ge 2 ]; do
  CFG=$1; GIB=$2; shift 2
  for r in $(seq "$ROUNDS"); do
    for nw in $NWS; do
      printf "%s %s nw=%s " "$CFG" "$GIB" "$nw"
      env ${KNOB:-EC_MI355X_NW8}=$nw EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only "$CFG" \
        --gib "$GIB" --steps 40 --warmup 20 2>/dev/null | tail -1 || exit 1
    done
  done
done
