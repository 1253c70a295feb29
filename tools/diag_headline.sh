set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu > gpurun_out/diag_bind_$i.log 2>&1 || exit $?
  EC_BENCH_NOBIND=1 timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu > gpurun_out/diag_nobind_$i.log 2>&1 || exit $?
done
timeout -k 10 120 python -u bench.py --gpus 1 --steps 200 --warmup 5 --no-extra --no-cpu > gpurun_out/diag_steps200.log 2>&1 || exit $?
for f in gpurun_out/diag_*.log; do python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l)
print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
