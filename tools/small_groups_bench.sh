#!/bin/bash
# Mixed-pattern decode rate by pattern-group size (1 GiB, 16 masks):
# groups < 8 stripes run ec_combine_fine, >= 8 the tiled ec_combine.
set -u
python -u -c "import torch; print(torch.cuda.is_available())"   # first import pages the image in
for spec in mixed:4+2:15:1 mixed:4+2:15:2 mixed:4+2:15:4 mixed:4+2:15:8 mixed:8+4:16:1 mixed:8+4:16:4 mixed:8+4:16:8 mixed:16+4:16:1 mixed:16+4:16:8; do
  echo "[$(date +%T)] $spec"
  timeout -k 10 180 python -u bench.py --only $spec --gib 1 --steps 10 --warmup 2 2>&1 | tail -1 || exit 1
done
