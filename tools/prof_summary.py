#!/usr/bin/env python3
"""Summarise tools/profile.sh output into profiles/ (committed evidence).

For every config directory triple (<cfg>_trace, <cfg>_FETCH_SIZE,
<cfg>_WRITE_SIZE) it reports, for the coder's kernels only:
  * calls and average duration from rocprofv3 --kernel-trace --stats,
  * HBM bytes per launch from the PMC passes, corrected as
    MI355X_MICROARCH.md section HBM prescribes: FETCH_SIZE and WRITE_SIZE are
    in KiB; on gfx950 FETCH_SIZE counts exactly half of a wide streaming
    read, so read bytes = 2 * 1024 * FETCH_SIZE; write bytes = 1024 *
    WRITE_SIZE (exact for 16-B-per-lane stores).
Algorithmic bytes per launch: encode S*(1+n/k), decode 2*S.
With tools/profile.sh's WARM_MS (launches keep running that long before the
40 timed ones), a second duration column averages the last 40 launches of
the kernel from the kernel trace: the rate past the clock transient of the
first ~10 ms of load, beside the all-launch average of
rocprofv3 --stats.

Usage: tools/prof_summary.py gpurun_out/prof_r01 profiles/r01 [traffic.json]
"""
import csv
import glob
import json
import os
import sys

OURS = ("ec_jit_combine", "ec_combine", "ec_encode_vander", "ec_encode_tile", "ec_slots")


def short(name):
    for o in OURS:
        if o in name:
            return name[name.index(o):].split("(")[0]
    return None


def stats(d):
    out = {}
    for row in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        s = short(row["Name"])
        if s:
            out[s] = dict(calls=int(row["Calls"]), avg_ns=float(row["AverageNs"]),
                          min_ns=float(row["MinNs"]), max_ns=float(row["MaxNs"]))
    return out


def tail_avg_ns(d, kern, last=40):
    """average duration of the kernel's last `last` launches (kernel trace)"""
    p = os.path.join(d, "run_kernel_trace.csv")
    if not os.path.exists(p):
        return None, 0
    rows = []
    for r in csv.DictReader(open(p)):
        if short(r["Kernel_Name"]) == kern:
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    rows = rows[-last:]
    if not rows:
        return None, 0
    return sum(e - b for b, e in rows) / len(rows), len(rows)


def counter(d, cname):
    vals = {}
    for row in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        s = short(row["Kernel_Name"])
        if s and row["Counter_Name"] == cname:
            vals.setdefault(s, []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def algorithmic(cfg, gib):
    kind, geo = cfg.split("_")[0], cfg.split("_")[1]
    k, r = map(int, geo.split("p"))
    S = int(gib * (1 << 30)) // (512 * k) * 512 * k
    if kind == "enc":
        return S, S * (k + k + r) // k
    if kind == "heal":
        return S, S + S * r // k
    if kind == "rmw":                       # user bytes in + n fragments out
        return S, S + S * (k + r) // k
    return S, 2 * S


def main():
    src, dst = sys.argv[1], sys.argv[2]
    traffic_path = sys.argv[3] if len(sys.argv) > 3 else None
    # GiB per config as tools/gpu_final.sh passes them
    gib = {"dec_4p2_3C": 1, "enc_4p2": 1, "enc_8p4": 0.25, "dec_8p4_FF0": 0.25,
           "enc_16p4": 2, "dec_8p4_EB5": 0.25, "dec_4p2_0F": 1, "mixed_8p4": 1, "heal_8p4": 1,
           "dec_16p4_FFFF0": 1, "mixed_16p4_64": 1, "rmw_4p2": 1, "rmw_8p4": 1, "rmw_16p4": 1}
    # overrides: PROF_GIB="dec_8p4_FF0=1,..." (a config profiled at another size)
    for kv in filter(None, os.environ.get("PROF_GIB", "").split(",")):
        name, val = kv.split("=")
        gib[name] = float(val)
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    lines = ["# rocprofv3 summary (%s)" % os.path.basename(src.rstrip("/")), "",
             "| config | kernel | calls | avg us (all) | user GB/s | algorithmic GB/s | HBM frac "
             "(8 TB/s) | avg us, last 40 | HBM frac, last 40 | PMC read MB | PMC write MB | "
             "PMC/algorithmic |",
             "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for tdir in sorted(glob.glob(os.path.join(src, "*_trace"))):
        cfg = os.path.basename(tdir)[:-len("_trace")]
        st = stats(tdir)
        fs = counter(tdir.replace("_trace", "_FETCH_SIZE"), "FETCH_SIZE")
        ws = counter(tdir.replace("_trace", "_WRITE_SIZE"), "WRITE_SIZE")
        S, alg = algorithmic(cfg, gib.get(cfg, 1))
        # the dominant kernel of the config = the one with most total time
        kern = max(st, key=lambda k: st[k]["calls"] * st[k]["avg_ns"])
        # encode configs also run one decode for the parity check
        if cfg.startswith("enc"):
            kern = next((k for k in st if "encode" in k), kern)
        elif cfg.startswith("rmw"):
            kern = next((k for k in st if "rmw" in k and "gather" not in k), kern)
        elif cfg.startswith("mixed") and any(k.startswith("ec_slots") for k in st):
            # sorted-slot groups: the tile kernel after the sort kernels
            kern = max((k for k in st if k.startswith("ec_combine")),
                       key=lambda k: st[k]["calls"] * st[k]["avg_ns"])
        elif any(k.startswith("ec_combine") for k in st):
            # the timed combine launches dominate the one setup encode
            kern = max((k for k in st if k.startswith("ec_combine")),
                       key=lambda k: st[k]["calls"])
        s = st[kern]
        rd = fs.get(kern, 0) * 1024 * 2
        wr = ws.get(kern, 0) * 1024
        t = s["avg_ns"] / 1e9
        tail, ntail = tail_avg_ns(tdir, kern)
        tail_cols = ("%.1f | %.3f" % (tail / 1e3, alg / (tail / 1e9) / 8e12)) if tail else "- | -"
        lines.append("| %s | `%s` | %d | %.1f | %.0f | %.0f | %.3f | %s | %.1f | %.1f | %.3f |" % (
            cfg, kern, s["calls"], s["avg_ns"] / 1e3, S / t / 1e9, alg / t / 1e9,
            alg / t / 8e12, tail_cols, rd / 1e6, wr / 1e6, (rd + wr) / alg))
        traffic[cfg] = dict(kernel=kern, avg_ns=s["avg_ns"], tail_avg_ns=tail, tail_launches=ntail,
                            user_bytes=S,
                            algorithmic_bytes=alg, hbm_read_bytes=rd, hbm_write_bytes=wr,
                            hbm_bytes_per_launch=rd + wr)
    lines += ["", "PMC correction: read = 2 x 1024 x FETCH_SIZE (gfx950 counts half of a "
              "wide streaming read), write = 1024 x WRITE_SIZE (MI355X_MICROARCH.md, HBM)."]
    open(dst + "_summary.md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))
    if traffic_path:
        # provenance of every entry: the profile, the commit
        # the profiled tree was at (this runs in the git checkout, after the
        # GPU run merged its output back) and when it was summarised
        import datetime
        import subprocess
        try:
            commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                                    text=True, cwd=os.path.dirname(os.path.abspath(__file__))
                                    ).stdout.strip() or None
        except OSError:
            commit = None
        prov = dict(profile=os.path.basename(src.rstrip("/")), summary=dst + "_summary.md",
                    commit=os.environ.get("PROF_COMMIT", commit),
                    date=datetime.date.today().isoformat())
        keymap = {"dec_4p2_3C": "dec_4+2_0x3C_1GiB"}
        tj = {keymap.get(k, k): dict(v, source=prov) for k, v in traffic.items()}
        json.dump(tj, open(traffic_path, "w"), indent=1)


if __name__ == "__main__":
    main()
