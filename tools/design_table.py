#!/usr/bin/env python3
"""Regenerate DESIGN.md's N=1 numbers table from one tools/gpu_round_end.sh
run: python3 tools/design_table.py TAG   (reads gpurun_out/TAG_bench.log,
profiles/TAG_summary.md and gpurun_out/prof_bench_TAG)."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag):
    b = json.loads(open(os.path.join(ROOT, "gpurun_out", tag + "_bench.log")).read()
                   .strip().split("\n")[-1])
    ex = b["extra"]
    summ = {}
    for l in open(os.path.join(ROOT, "profiles", tag + "_summary.md")):
        if l.startswith("| ") and not l.startswith("| config"):
            c = [x.strip() for x in l.strip().strip("|").split("|")]
            summ[c[0]] = c
    stats = glob.glob(os.path.join(ROOT, "gpurun_out", "prof_bench_" + tag, "**",
                                   "*kernel_stats.csv"), recursive=True)
    head_calls, head_avg = 0, 0.0
    for r in csv.DictReader(open(stats[0])):
        if "ec_combine<4, 1, 8" in r["Name"]:
            head_calls, head_avg = int(r["Calls"]), float(r["AverageNs"]) / 1e3

    def R(cfg):
        c = summ.get(cfg)
        return (c[3], c[6], c[9]) if c else ("", "", "")

    def E(key, f="user_GBps"):
        return ex[key][f]

    rows = [
        ("**4+2 decode, mask 0x3C, 1 GiB (headline, BASELINE configs[1])**",
         "**%.0f**" % b["value"], "**%.3f**" % b["roofline"]["frac"], R("dec_4p2_3C")),
        ("the same, sustained (50 launches after 150 ms of back-to-back launches)",
         "%.0f" % E("dec_4+2_0x3C_1GiB_sustained"),
         "%.3f" % E("dec_4+2_0x3C_1GiB_sustained", "hbm_frac"), ("", "", "")),
    ]
    for name, key, cfg in (
            ("4+2 decode, mask 0x0F, 1 GiB", "dec_4+2_0x0F_1GiB", None),
            ("4+2 encode, 1 GiB", "enc_4+2_1GiB", "enc_4p2"),
            ("8+4 encode, 64K-stripe batch (configs[2])", "enc_8+4_64Kstripes", "enc_8p4"),
            ("8+4 decode 0xFF0, 64K-stripe batch", "dec_8+4_0xFF0_64Kstripes", "dec_8p4_FF0"),
            ("8+4 decode 0xEB5, 64K-stripe batch", "dec_8+4_0xEB5_64Kstripes", None),
            ("8+4 decode 0xFF0, 1 GiB", "dec_8+4_0xFF0_1GiB", None),
            ("16+4 encode, 2 GiB (configs[3] slice)", "enc_16+4_2GiB", "enc_16p4"),
            ("16+4 decode 0xFFFF0, 1 GiB", "dec_16+4_0xFFFF0_1GiB", "dec_16p4_FFFF0"),
            ("self-heal, 8+4, 16 masks, 1024-stripe groups (configs[4] slice)",
             "selfheal_mixed16_8+4_1GiB", "mixed_8p4"),
            ("self-heal, 16+4, 64 masks (device table)", "selfheal_mixed64_16+4_1GiB",
             "mixed_16p4_64"),
            ("fused heal 8+4, regenerate 4 fragments", "heal_fused_8+4_regen4_1GiB", "heal_8p4"),
            ("partial write 4+2, 1 GiB at an odd address", "writev_rmw_4+2_1GiB_unaligned",
             "rmw_4p2")):
        rows.append((name, "%.0f" % E(key), "%.3f" % E(key, "hbm_frac"),
                     R(cfg) if cfg else ("", "", "")))
    e = ex["e2e_pcie_4+2_512MiB"]
    ce = ex["cpu_engine_4+2_1GiB"]
    cb = b["cpu_baseline"]
    lines = ["| config | bench user GB/s | bench of peak | rocprof µs | rocprof of peak | "
             "PMC / algorithmic |", "|---|---|---|---|---|---|"]
    for name, u, f, (us, rf, pm) in rows:
        lines.append("| %s | %s | %s | %s | %s | %s |" % (name, u, f, us, rf, pm))
    lines.append("| PCIe-inclusive, pinned host buffers, 4+2 enc / dec 512 MiB | %.1f / %.1f | "
                 "(link-bound) | | | |" % (e["enc_user_GBps"], e["dec_user_GBps"]))
    lines.append("| CPU engine (AVX-512), 16 threads, 4+2 enc / dec 1 GiB (1 thread: %.1f / %.1f) "
                 "| %.1f / %.1f | | | | |" % (ce["one_thread_encode_GBps"],
                                           ce["one_thread_decode_GBps"], ce["encode_GBps"],
                                           ce["decode_GBps"]))
    lines.append("| `cpu_baseline`: oracle (portable-C class), 16 threads, 4+2 decode / configs[0] "
                 "encode (1 thread: %.1f / %.1f) | %.1f / %.1f | | | | |" % (
                     cb["one_thread_decode_GBps"], cb["one_thread_encode_GBps"], cb["value"],
                     cb["encode_1GiB_GBps"]))
    head = ('Latest N=1 numbers (MI355X, HEAD of round 2, `tools/gpu_round_end.sh`, tag `%s`). '
            '"bench" = `bench.py --gpus 1 --steps 20 --warmup 5` event timing '
            '(`profiles/%s/%s_bench.log`; `extra` configs 10 launches after 20); the same '
            'command\'s headline under `rocprofv3 --kernel-trace --stats` (`--no-extra --no-cpu`, '
            '`profiles/%s/bench_rocprof_kernel_stats.csv`): %d launches of the headline kernel '
            'averaging %.1f µs against the bench\'s %.1f µs event average. "rocprof" columns = '
            'average over 50 launches per config (`profiles/%s_summary.md`, `profiles/%s_prof/`), '
            'with PMC HBM bytes against algorithmic bytes. Of peak = algorithmic bytes / time / '
            '8 TB/s. Earlier boxes this round: `profiles/r02_end_summary.md`, '
            '`profiles/r02z2_summary.md`, `profiles/r02z_summary.md`.\n\n' % (
                tag, tag, tag, tag, head_calls, head_avg, b["roofline"]["avg_launch_ms"] * 1e3,
                tag, tag))
    p = os.path.join(ROOT, "DESIGN.md")
    s = open(p).read()
    a = s.index("Latest N=1 numbers (MI355X, HEAD of round 2")
    z = s.index("The rocprof averages include the warm-up launches")
    s = s[:a] + head + "\n".join(lines) + "\n\n" + s[z:]
    open(p, "w").write(s)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1])
