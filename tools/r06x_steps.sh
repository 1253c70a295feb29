# round-6 GPU call: the 16+4 host encode as a combine, by the persistent
# grid's input in flight (EC_ZC_INFLIGHT_KB), beside the register encoder
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] zc_sizes"
for r in 1 2; do for c in "0 2048" "1 2048" "1 4096" "1 8192"; do set -- $c
  EC_GPU_ALWAYS=1 EC_MI355X_ZCENC16=$1 EC_ZC_INFLIGHT_KB=$2 ZC_GEOS="16+4" ZC_SIZES="32 64 256 512" timeout -k 10 300 python3 tools/zc_sizes.py >> gpurun_out/r06x_zcsizes.log 2>&1 || { tail -20 gpurun_out/r06x_zcsizes.log; exit 1; }
done; done
grep -E "^16\+4" gpurun_out/r06x_zcsizes.log | sed -E 's/heal.*\[/[/; s/EC_MI355X_ZCDB=unset EC_ZC_TPB=unset //'
echo "[$(date +%T)] done"
