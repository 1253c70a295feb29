# Tile order A/B for the tile encoders (EC_MI355X_TILE_PERM=1: golden-ratio
# order), with the fragment placements of tools/placeab.sh.
set -u
mkdir -p gpurun_out
TAG=${TAG:-r05as}
{
timeout -k 10 300 env ${PERM_VAR:-EC_MI355X_TILE_PERM}=${PARITY_PERM:-1} python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "${PARITY_K:-encode or fullsize}" || exit 1
for r in 1 2 3; do
 IFS=, read -ra CASES <<< "${PERM_CASES:-enc:16+4 8 0,enc:16+4 8 4096,enc:16+4 2 0,enc:16+4 2 4096,enc:4+2 1 0,enc:8+4 2 0}"
 for c in "${CASES[@]}"; do
  set -- $c
  for pm in ${PERMS:-0 1}; do
   echo "== round $r $1 $2 GiB stagger $3 perm $pm"
   timeout -k 10 120 env ${PERM_VAR:-EC_MI355X_TILE_PERM}=$pm EC_BENCH_FRAG_STAGGER=$3 python3 bench.py --only $1 --gib $2 --steps 20 --warmup 5 --warm-ms 150 || exit 1
  done
 done
done
} > gpurun_out/${TAG}_permab.log 2>&1
