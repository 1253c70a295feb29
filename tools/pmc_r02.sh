#!/bin/bash
# PMC counters of one product kernel driven by bench.py --only, one
# rocprofv3 --pmc pass per counter set (<= 8 SQ counters each).
# Usage: tools/pmc_r02.sh TAG CONFIG GIB
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; CFG=$2; GIB=$3
cd /tmp && export TMPDIR=/tmp
i=0
for C in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVES" \
         "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"; do
  i=$((i+1))
  echo "[$(date +%T)] pass $i: $C"
  timeout -s KILL 120 rocprofv3 --kernel-trace --kernel-include-regex ec_ --pmc $C -d $R/gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- \
    python3 $R/bench.py --only "$CFG" --gib "$GIB" --steps 5 --warmup 1 > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || exit 1
  python3 $R/tools/prof_filter.py $R/gpurun_out/pmc_${TAG}_$i
done
