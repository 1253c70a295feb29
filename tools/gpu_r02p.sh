#!/bin/bash
# Full validation pass: every GPU test, smoke(), the default bench line and a
# rocprof kernel trace of the headline bench.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r02p}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -3 "gpurun_out/${TAG}_$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
run smoke 200 python3 -c "import __graft_entry__ as e; e.smoke()"
run bench 700 python -u bench.py
run bench_rocprof 600 bash -c 'cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench_'$TAG' -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-extra --no-cpu && python3 $GRAFT_REPO_ROOT/tools/prof_filter.py $GRAFT_REPO_ROOT/gpurun_out/prof_bench_'$TAG' ecdev'
du -sh gpurun_out
