#!/bin/bash
# SQ counters of the k = 16 decode and its compute-only / no-load / no-store
# probes (tools/kbench/kb3.hip group probe16), one rocprofv3 --pmc pass per
# counter set.  Usage (GPU box): tools/pmc_probe16.sh TAG
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-probe16}
i=0
for C in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_IFETCH SQC_ICACHE_MISSES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "kb_combine_probe|ec_combine" \
    -d $R/gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- \
    $R/tools/kbench/kb3 1 3 probe16 > $R/gpurun_out/pmc_${TAG}_$i.log 2>&1 || exit 1
  echo "pass $i done"
done
