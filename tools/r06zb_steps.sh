# round-6 GPU call: partial-write staging from 16-byte-aligned loads (SM=8)
# against the shipped dword-aligned shift staging (SM=3), interior +3 / +7 /
# +13 bytes, kb3 group rmw
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] kb3"
timeout -k 10 500 tools/kbench/kb3_r06 1 7 rmw > gpurun_out/r06zb_kb3_rmw.log 2>&1 || { tail -20 gpurun_out/r06zb_kb3_rmw.log; exit 1; }
cat gpurun_out/r06zb_kb3_rmw.log
echo "[$(date +%T)] done"
