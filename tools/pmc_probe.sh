#!/bin/bash
# Development probe (not product): SQ/SQC counters of the kbench2 kernels,
# one rocprofv3 --pmc pass per counter set.  Usage: tools/pmc_probe.sh TAG
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=${1:-probe}
i=0
for C in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_BRANCH" \
         "SQC_ICACHE_MISSES SQ_WAIT_INST_LDS SQ_IFETCH SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- \
    $R/tools/kbench/kbench2 1 2 > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || exit 1
done
