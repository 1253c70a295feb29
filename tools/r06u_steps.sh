# round-6 GPU call: same-box A/B of the device-table change through
# bench.py --only (base = 9df9427, the pattern parked in LDS; head = scalar
# loads), alternating processes, 3 rounds, 150 ms of load before 40 launches
set -u
mkdir -p gpurun_out
echo "[$(date +%T)] ablib"
AB_LIBS="base=glusterfs_amd/lib_ab6/libec_mi355x_base.so head=" timeout -k 10 900 bash tools/ab_lib.sh 'mixed:16+4:64 1 mixed:8+4 1' > gpurun_out/r06u_ablib_mixed.log 2>&1 || { tail -20 gpurun_out/r06u_ablib_mixed.log; exit 1; }
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/r06u_ablib_mixed.log") if l.startswith("{")]
for r in rows:
    res=r["res"]
    print(r["round"], r["lib"], res.get("only"), res.get("kernel_ms"), res.get("ok"))
PY
echo "[$(date +%T)] done"
