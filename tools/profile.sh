#!/bin/bash
# rocprofv3 profiles of the dominant kernels (run on the GPU box via gpurun).
# Pass 1: --kernel-trace --stats; passes 2/3: PMC FETCH_SIZE and WRITE_SIZE
# (separate passes: they do not fit one TCC slot set, MI355X_MICROARCH.md).
# Usage: tools/profile.sh TAG CONFIG GIB [CONFIG GIB ...]
#   CONFIG = dec:4+2:3C | enc:4+2 | enc:8+4 | dec:8+4:FF0 ...
# WARM_MS=150: launches keep running that long before the 40 timed ones (the
# trace then holds the warm-up launches too: tools/trace_seq.py LAST=40 gives
# the average over the timed tail)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
while [ $# -ge 2 ]; do
  CFG=$1; GIB=$2; shift 2
  NAME=$(echo "$CFG" | tr ':+' '_p')
  for PASS in trace FETCH_SIZE WRITE_SIZE; do
    if [ $PASS = trace ]; then ARGS="--kernel-trace --stats"; else ARGS="--kernel-trace --kernel-include-regex ec_ --pmc $PASS"; fi
    echo "[$(date +%T)] $CFG $PASS"
    timeout -k 10 300 rocprofv3 $ARGS -d "$OUT/${NAME}_$PASS" -o run --output-format csv -- \
      python3 "$R/bench.py" --only "$CFG" --gib "$GIB" --steps 40 --warmup 10 --warm-ms "${WARM_MS:-0}" \
      > "$OUT/${NAME}_$PASS.log" 2>&1
    rc=$?
    echo "rc=$rc"; tail -2 "$OUT/${NAME}_$PASS.log"
    if [ $rc -ne 0 ]; then exit $rc; fi
    python3 "$R/tools/prof_filter.py" "$OUT/${NAME}_$PASS"
  done
done
