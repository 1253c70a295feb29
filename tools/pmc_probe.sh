cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export KB_K=16
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_IFETCH SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/pmc16_$i -o run --output-format csv -- $R/tools/kbench/kbench2 1 2 > $R/gpurun_out/pmc16_$i.log 2>&1 || exit 1
done
