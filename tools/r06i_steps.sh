# round-6 GPU call: kernel durations of the k = 16 decode under rocprof in the
# bench's own process (torch allocations), JIT off / on
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in 0 1 0 1; do
  echo "[$(date +%T)] jit=$v"
  EC_MI355X_JIT=$v EC_MI355X_JIT_SYNC=1 EC_MI355X_QUIET=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r06i_jit$v -o run --output-format csv -- python3 $R/bench.py --only dec:16+4:FFFF0 --gib 1 --steps 40 --warmup 10 --warm-ms 150 > $R/gpurun_out/r06i_jit$v.log 2>&1 || exit 1
  tail -1 $R/gpurun_out/r06i_jit$v.log
  python3 - "$R/gpurun_out/prof_r06i_jit$v" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "ec_" in row["Name"]:
            print("%-70s calls %5s avg %9.1f us min %9.1f" % (row["Name"][:70], row["Calls"], float(row["AverageNs"]) / 1e3, float(row["MinNs"]) / 1e3))
PY
done
echo "[$(date +%T)] done"
