#!/bin/bash
# Clocks, power and temperature beside a long run of back-to-back headline
# decodes (does the sustained slowdown follow sclk, mclk or power?).
# rocm-smi sampled every ~0.25 s into a file while rocprofv3 traces every
# launch of 3000 x 1 GiB 4+2 decodes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sustain_clk
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
( for i in $(seq 120); do
    echo "T $(date +%s.%N)"
    rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "^GPU\[0\]" | grep -E "sclk|mclk|fclk|Power|Temperature" || true
    sleep 0.2
  done ) > "$OUT/smi.txt" 2>&1 &
SMI=$!
sleep 1
timeout -k 10 120 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --only dec:4+2:3C --gib 1 --steps 3000 --warmup 2 > "$OUT/bench.log" 2>&1
rc=$?
sleep 2
kill $SMI 2>/dev/null
wait $SMI 2>/dev/null
python3 "$R/tools/prof_filter.py" "$OUT/trace" ec_combine
python3 - "$OUT" <<'PY'
import csv, glob, sys
o = sys.argv[1]
f = glob.glob(o + "/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "ec_combine<4, 1, 8" in r["Kernel_Name"]]
t0 = int(rows[0]["Start_Timestamp"])
with open(o + "/durations.txt", "w") as fh:
    for r in rows:
        fh.write("%.3f %.1f\n" % ((int(r["Start_Timestamp"]) - t0) / 1e6,
                                  (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
n = len(rows)
for a, b in ((0, 20), (20, 100), (100, 500), (500, 1500), (1500, n)):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows[a:b]]
    if d:
        print("launches %d-%d: mean %.1f us, min %.1f, max %.1f" % (a, b, sum(d) / len(d), min(d), max(d)))
PY
exit $rc
