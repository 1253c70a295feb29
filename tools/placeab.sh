# Fragment placement A/B (bench.py EC_BENCH_FRAG_STAGGER): the n fragment
# buffers as separate torch allocations (0) or as views of one allocation
# whose bases sit `stagger` bytes off multiples of the fragment size.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r05ar}
{
for r in 1 2 3; do
 IFS=, read -ra CASES <<< "${PLACE_CASES:-enc:16+4 8,enc:16+4 2,dec:4+2:3C 1,enc:4+2 1}"
 for c in "${CASES[@]}"; do
  set -- $c
  for st in ${STAGGERS:-0 256 4096 2162688}; do
   echo "== round $r $1 $2 GiB stagger $st"
   timeout -k 10 120 env EC_BENCH_FRAG_STAGGER=$st python3 bench.py --only $1 --gib $2 --steps 20 --warmup 5 --warm-ms 150 || exit 1
  done
 done
done
} > gpurun_out/${TAG}_placeab.log 2>&1
