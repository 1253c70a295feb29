#!/bin/bash
# Same-box A/B of builds of the library through bench.py --only:
# alternating processes, ROUNDS rounds, one JSON line per (round, build, config).
#   tools/ab_lib.sh 'mixed:8+4 1 dec:8+4:FF0 1'
# Builds: AB_LIBS="name=path ..." (path empty = the in-tree lib/libec_mi355x.so),
# default "base=glusterfs_amd/lib_ab/libec_mi355x_base.so head=" (other
# builds: a `make` of another commit's glusterfs_amd, copied to lib_ab/).
set -u
LIBS=${AB_LIBS:-"base=glusterfs_amd/lib_ab/libec_mi355x_base.so head="}
ROUNDS=${ROUNDS:-3}
set -- $1
for r in $(seq 1 "$ROUNDS"); do
  for spec in $LIBS; do
    name=${spec%%=*}; path=${spec#*=}
    if [ -n "$path" ]; then L=$PWD/$path; else L=; fi
    for ((i = 1; i <= $#; i += 2)); do
      cfg=${!i}; j=$((i + 1)); gib=${!j}
      out=$(EC_MI355X_LIB=$L EC_MI355X_QUIET=1 timeout -k 10 120 python3 bench.py --only "$cfg" \
            --gib "$gib" --steps 40 --warmup 10 --warm-ms "${WARM_MS:-150}" 2>/dev/null | grep '^{') || exit 1
      echo "{\"round\": $r, \"lib\": \"$name\", \"res\": $out}"
    done
  done
done
