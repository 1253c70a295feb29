#!/bin/bash
# PMC of the 16+4 partial-write encoder (ec_encode_tile_rb<...,SM=1>: the
# interior read in place at the caller's byte offset) beside the aligned
# 16+4 encoder (SM=0), same launches, one rocprofv3 --pmc pass per counter
# set.  Also lists the counters the box offers.
# Usage (GPU box): tools/pmc_rmw16.sh TAG ["SET1" "SET2" ...]
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-rmw16}
shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || echo "counter listing failed"
if [ $# -eq 0 ]; then
  set -- "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU" \
         "SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
fi
i=0
for C in "$@"; do
  i=$((i+1))
  for CFG in rmw:16+4 enc:16+4; do
    NAME=$(echo "$CFG" | tr ':+' '_p')
    timeout -s KILL 90 rocprofv3 --pmc $C --kernel-include-regex "ec_encode_tile" \
      -d "$OUT/${NAME}_$i" -o run --output-format csv -- \
      python3 "$R/bench.py" --only "$CFG" --gib 1 --steps 20 --warmup 5 > "$OUT/${NAME}_$i.log" 2>&1 || exit 1
    echo "pass $i $CFG done"
  done
done
