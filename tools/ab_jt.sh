#!/bin/bash
# Same-box A/B of the multiply dispatch (switch / jump table / row block)
# through the product launcher: alternating processes, EC_MI355X_JT in $JTS
# (default "0 1"), bench --only.
# Usage: [JTS="1 3"] tools/ab_jt.sh ROUNDS CONFIG GIB [CONFIG GIB ...]
set -u
ROUNDS=$1; shift
while [ $# -ge 2 ]; do
  CFG=$1; GIB=$2; shift 2
  for r in $(seq "$ROUNDS"); do
    for jt in ${JTS:-0 1}; do
      printf "%s jt=%s " "$CFG" "$jt"
      EC_MI355X_JT=$jt EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only "$CFG" \
        --gib "$GIB" --steps "${STEPS:-20}" --warmup "${WARMUP:-3}" || exit 1
    done
  done
done
