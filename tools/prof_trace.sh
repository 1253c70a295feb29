#!/bin/bash
# rocprofv3 kernel-trace + stats of `bench.py --only CONFIG` runs (no PMC).
# Usage: tools/prof_trace.sh TAG CONFIG GIB [CONFIG GIB ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
while [ $# -ge 2 ]; do
  CFG=$1; GIB=$2; shift 2
  NAME=$(echo "$CFG" | tr ':+' '_p')
  echo "[$(date +%T)] $CFG"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$NAME" -o run --output-format csv -- \
    python3 "$R/bench.py" --only "$CFG" --gib "$GIB" --steps ${STEPS:-10} --warmup 2 > "$OUT/$NAME.log" 2>&1
  rc=$?
  echo "rc=$rc"; tail -1 "$OUT/$NAME.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
  python3 "$R/tools/prof_filter.py" "$OUT/$NAME"
  grep -h "ec_" "$OUT/$NAME"/*kernel_stats.csv | cut -c1-200
  python3 "$R/tools/trace_seq.py" "$OUT/$NAME" > "$OUT/${NAME}_seq.txt"
done
