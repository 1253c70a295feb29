#!/bin/bash
# One gpurun call running a chosen list of steps at HEAD, each under its own
# time limit, stopping at the first failure (no retries):
#   TAG=r03a tools/gpu_steps.sh smoke pytest bench
# Steps: smoke | pytest | pytest_new (the files in $TESTS) | bench | bench_rocprof
#        | rehearsal (2 gloo ranks on GPU 0) | profile (per-config rocprof + PMC)
#        | kbench (tools/kbench/kbench $KBENCH_ARGS) | kb3 (tools/kbench/kb3 $KB3_ARGS)
#        | zcab (heal sweep, zero-copy combine A/B) | zcsizes (pinned decodes 4-256 MiB, A/B) | zcheal (pinned 16+4 / 8+4 decode, encode, heal, row-masked encode, ZCDB A/B) | fuzz (tools/fuzz_api.py: random calls of every entry point and buffer kind against the oracle, GPU-always then auto) | fuzzjit (device buffers only, the run-time compiled kernels from 16 stripes up) | pcie (DMA copy ceiling of the link, each way and duplex) | zctpb (pinned decodes + encodes 1-256 MiB by EC_ZC_TPB / EC_ZC_INFLIGHT_KB) | hsweep (kernel trace of the 4 MiB heal sweep, GPU engine) | hostlat (host cost of one device call) | hsweep3 (heal sweep by buffer provenance, auto / gpu / cpu) | ablib (tools/ab_lib.sh: two library builds alternating through bench.py --only) | concur (tools/kbench/concur: concurrent vs coalesced-ceiling calls, auto / gpu / cpu) | sharesweep (heal sweep, auto, split share fixed per mille; 0 = the model's) | busyab (heal windows on $BUSY_BUFS buffers from 2/4/8 threads, the busy-staging rule off / on, and CPU-only) | trace (per-launch rocprof sequence, STEPS launches of $TRACE_ARGS)
# Logs go to gpurun_out/${TAG}_<step>.log.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -4 "gpurun_out/${TAG}_$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    pytest_new) run pytest_new 600 python -u -m pytest ${TESTS} -m gpu -x -v --timeout 120 --timeout-method thread ;;
    bench) run bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench_rocprof) run bench_rocprof 300 bash -c "cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench_$TAG -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-extra --no-cpu && python3 $R/tools/prof_filter.py $R/gpurun_out/prof_bench_$TAG ec_" ;;
    rehearsal) run rehearsal 300 env EC_BENCH_BACKEND=gloo EC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 1 ;;
    rehearsal4) run rehearsal4 600 env EC_BENCH_BACKEND=gloo EC_BENCH_DEVICE=0 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 4 --steps 3 --warmup 1 ;;
    profile) run profile 900 bash tools/profile.sh "$TAG" ${PROFILE_ARGS:-dec:4+2:3C 1 enc:4+2 1 enc:8+4 0.25 dec:8+4:FF0 0.25 enc:16+4 2 mixed:8+4 1 heal:8+4 1 dec:16+4:FFFF0 1 mixed:16+4:64 1 rmw:4+2 1 rmw:8+4 1 rmw:16+4 1} ;;
    kbench) run kbench 600 tools/kbench/kbench ${KBENCH_ARGS:-} ;;
    trace) run trace 600 bash tools/prof_trace.sh "$TAG" ${TRACE_ARGS:-dec:16+4:FFFF0 1 dec:4+2:3C 1} ;;
    zcab) run zcab 600 bash -c 'for r in 1 2 3; do for v in 0 1; do echo "== round $r EC_MI355X_ZCDB=$v"; EC_GPU_ALWAYS=1 EC_MI355X_ZCDB=$v python3 bench.py --heal-sweep gpu --steps 256 || exit 1; done; done' ;;
    zcsizes) run zcsizes 600 bash -c 'for r in 1 2; do for v in 0 1; do EC_GPU_ALWAYS=1 EC_MI355X_ZCDB=$v python3 tools/zc_sizes.py || exit 1; done; done' ;;
    zctpb) run zctpb 900 bash -c 'for r in 1 2; do for c in "0 2048" "4 2048" "0 1024" "0 4096"; do set -- $c; EC_GPU_ALWAYS=1 EC_ZC_TPB=$1 EC_ZC_INFLIGHT_KB=$2 ZC_SIZES="${ZC_SIZES:-1 2 4 8 16 64 256}" python3 tools/zc_sizes.py || exit 1; done; done' ;;
    zcheal) run zcheal 600 bash -c 'for r in 1 2; do for v in 0 1; do EC_GPU_ALWAYS=1 EC_MI355X_ZCDB=$v ZC_GEOS="16+4 8+4" ZC_SIZES="4 16 64" python3 tools/zc_sizes.py || exit 1; done; done' ;;
    fuzz) run fuzz $(( ${FUZZ_SECS:-150} + 300 )) bash -c 'EC_GPU_ALWAYS=1 FUZZ_SECS=${FUZZ_SECS:-150} python3 -u tools/fuzz_api.py && EC_GPU_ALWAYS=0 FUZZ_SECS=60 python3 -u tools/fuzz_api.py' ;;
    fuzzjit) run fuzzjit $(( ${FUZZ_SECS:-120} + 200 )) bash -c 'EC_GPU_ALWAYS=1 EC_MI355X_JIT_MIN_STRIPES=16 FUZZ_KINDS="device device_offset" FUZZ_SECS=${FUZZ_SECS:-120} python3 -u tools/fuzz_api.py' ;;
    rmwab) run rmwab 600 bash -c 'export EC_GPU_ALWAYS=1 FUZZ_THREADS=12 FUZZ_SECS=${FUZZ_SECS:-100} FUZZ_KINDS="device device_offset" FUZZ_OPS="writev decode encode stream_chain"; echo "== default (LDS-DMA at the caller alignment)"; python3 -u tools/fuzz_api.py; a=$?; echo "== EC_MI355X_ENC=0 (register encoders, aligned loads + alignbyte)"; EC_MI355X_ENC=0 python3 -u tools/fuzz_api.py; b=$?; echo "rc default=$a enc0=$b"' ;;
    regrepro) run regrepro 600 env EC_GPU_ALWAYS=1 python3 -u tools/reg_repro.py ${REPRO_ITERS:-60} ;;
    pcie) run pcie 200 bash -c 'for m in 4 16 256; do python3 tools/pcie_probe.py $m || exit 1; done' ;;
    hsweep) run hsweep 300 bash -c "cd /tmp && export TMPDIR=/tmp && EC_GPU_ALWAYS=1 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_hsweep_$TAG -o run --output-format csv -- python3 $R/bench.py --heal-sweep gpu --steps 64 && python3 $R/tools/prof_filter.py $R/gpurun_out/prof_hsweep_$TAG ec_ && python3 $R/tools/trace_seq.py $R/gpurun_out/prof_hsweep_$TAG" ;;
    hostlat) run hostlat 180 python -u tools/host_latency.py ;;
    concur) run concur 400 bash -c 'EC_GPU_ALWAYS=0 tools/kbench/concur ${CONCUR_SECS:-1} auto && EC_GPU_ALWAYS=1 tools/kbench/concur ${CONCUR_SECS:-1} auto && EC_GPU_ALWAYS=0 tools/kbench/concur ${CONCUR_SECS:-1} avx' ;;
    busyab) run busyab 600 bash -c 'for r in 1 2; do for t in ${BUSY_THREADS:-2 4 8}; do for c in 0 10; do echo "== round $r threads $t EC_STAGE_COPY_GBPS=$c"; EC_GPU_ALWAYS=0 EC_STAGE_COPY_GBPS=$c CONCUR_HEAL_THREADS=$t CONCUR_SCEN=heal tools/kbench/concur 1 auto ${BUSY_BUFS:-pageable} || exit 1; done; echo "== round $r threads $t cpu"; EC_GPU_ALWAYS=0 CONCUR_HEAL_THREADS=$t CONCUR_SCEN=heal tools/kbench/concur 1 avx ${BUSY_BUFS:-pageable} || exit 1; done; done' ;;
    sharesweep) run sharesweep 900 bash -c 'for r in 1 2; do for f in ${SHARES:-0 350 450 550 650}; do echo "== round $r EC_HYBRID_SHARE=$f"; EC_GPU_ALWAYS=0 EC_HYBRID_SHARE=$f python3 bench.py --heal-sweep auto --steps 256 || exit 1; done; done' ;;
    hsauto) run hsauto 900 bash -c 'for r in ${HS_ROUNDS:-1 2 3}; do echo "== round $r"; EC_GPU_ALWAYS=0 python3 bench.py --heal-sweep auto --steps 256 || exit 1; done' ;;
    learnab) run learnab 900 bash -c 'for r in ${HS_ROUNDS:-1 2}; do for l in 0 1; do echo "== round $r EC_SPLIT_LEARN=$l"; EC_GPU_ALWAYS=0 EC_SPLIT_LEARN=$l python3 bench.py --heal-sweep auto --steps 256 || exit 1; done; done' ;;
    ablib) run ablib 900 bash tools/ab_lib.sh "${AB_ARGS:-mixed:8+4 1 mixed:16+4:64 1 dec:8+4:FF0 1}" ;;
    hsweep3) run hsweep3 400 bash -c 'for m in auto gpu cpu; do echo "== $m"; if [ $m = gpu ]; then E=1; else E=0; fi; EC_GPU_ALWAYS=$E python3 bench.py --heal-sweep $m --steps 256 || exit 1; done' ;;
    kb3) run kb3 600 tools/kbench/kb3 ${KB3_ARGS:-1 7 all} ;;
    sizes) run sizes 900 bash -c 'for r in 1 2; do for c in ${SIZE_CASES:-"enc:16+4 2" "enc:16+4 8" "dec:4+2:3C 1" "dec:4+2:3C 4" "enc:4+2 1" "enc:4+2 4"}; do set -- $c; echo "== round $r $1 $2 GiB"; python3 bench.py --only $1 --gib $2 --steps 20 --warmup 5 --warm-ms 150 || exit 1; done; done' ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$(date +%T)] done"
