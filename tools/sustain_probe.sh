#!/bin/bash
# Sustained-launch probe: per-launch kernel durations of 60 back-to-back
# launches (does a kernel slow down as the card heats / hits its power cap?),
# with rocm-smi clock / power readings before and after.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/sustain_${1:-x}
mkdir -p "$OUT"
shift
for CFG in "$@"; do
  NAME=$(echo "$CFG" | tr ':+' '_p')
  (rocm-smi --showpower --showtemp --showclocks 2>&1 | grep -E "^GPU\[0\]|Power|Temp|sclk|mclk|fclk" | head -12) > "$OUT/${NAME}_smi_before.txt" || true
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/$NAME" -o run --output-format csv -- \
    python3 "$R/bench.py" --only "$CFG" --gib 1 --steps 60 --warmup 2 > "$OUT/$NAME.log" 2>&1 || exit 1
  (rocm-smi --showpower --showtemp --showclocks 2>&1 | grep -E "^GPU\[0\]|Power|Temp|sclk|mclk|fclk" | head -12) > "$OUT/${NAME}_smi_after.txt" || true
  python3 "$R/tools/prof_filter.py" "$OUT/$NAME" ec_combine
  python3 - "$OUT/$NAME" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in csv.DictReader(open(f))]
print(sys.argv[1].split("/")[-1], "n=%d" % len(d), " ".join("%.0f" % x for x in d))
PY
done
