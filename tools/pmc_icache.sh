#!/bin/bash
# Instruction-cache PMC of the combine kernels (is the 16+4 decode's compute
# bound by fetches of the jump-table bodies?).  One counter set per pass.
# Usage: tools/pmc_icache.sh TAG CONFIG GIB [CONFIG GIB ...]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc_avail.txt 2>&1 || true
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_]*" $R/gpurun_out/pmc_avail.txt | sort -u > $R/gpurun_out/pmc_avail_sqc.txt || true
while [ $# -ge 2 ]; do
  CFG=$1; GIB=$2; shift 2
  N=$(echo "$CFG" | tr ':+' '_p')
  for C in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVE_CYCLES" \
           "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    P=$(echo "$C" | cut -d' ' -f1)
    echo "[$(date +%T)] $CFG: $C"
    timeout -s KILL 60 rocprofv3 --kernel-trace --kernel-include-regex ec_ --pmc $C -d $R/gpurun_out/pmcic_${TAG}_${N}_$P -o run --output-format csv -- \
      python3 $R/bench.py --only "$CFG" --gib "$GIB" --steps 5 --warmup 1 > $R/gpurun_out/pmcic_${TAG}_${N}_$P.log 2>&1 || exit 1
    python3 $R/tools/prof_filter.py $R/gpurun_out/pmcic_${TAG}_${N}_$P
  done
done
