#!/usr/bin/env python3
"""Benchmark of the MI355X disperse coder (BASELINE.json metric).

One "step" = one pass of the hot path over one batch resident in HBM:
decoding 1 GiB of user data of a disperse 4+2 volume with 2 fragments
missing (mask 0x3C: bricks 0 and 1 lost), i.e. BASELINE.json configs[1].
With --gpus N (one process per GPU under torch.distributed.run) every rank
decodes its own 1 GiB stripe range (weak scaling; stripes are independent,
no collective touches the data path -- the only collectives are the barrier
and the max-over-ranks of the timing).

Besides the headline line, the JSON carries:
  roofline      HBM roofline of the decode kernel (algorithmic bytes 2*S per
                launch / average launch time measured with HIP events on the
                launch stream; traffic from the committed rocprofv3 PMC run)
  cpu_baseline  the CPU oracle (oracle/, a C restatement of the reference
                algorithm) decoding a bounded sample of the same fragments on
                the host's cores, rank 0 at N=1 only
  extra         the other BASELINE configs measured the same way (4+2 and
                8+4 encode/decode device-resident, 16+4 encode, mixed-pattern
                self-heal decode, PCIe-inclusive end-to-end rates)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "EC encode/decode user-data GB/s (4+2, 8+4) at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CHUNK = 512


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--gib", type=float, default=1.0, help="user data per GPU per step")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--only", default=None, help="profile helper: run one config only")
    return ap.parse_args()


def rand_u8(torch, nbytes, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randint(-2**62, 2**62, (nbytes // 8,), dtype=torch.int64, device=device,
                      generator=g)
    return x.view(torch.uint8)


class Timer:
    """K launches between two HIP events on the launch stream."""

    def __init__(self, torch):
        self.torch = torch

    def run(self, fn, steps, warmup, barrier=None):
        torch = self.torch
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        if barrier:
            barrier()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for _ in range(steps):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if barrier:
            barrier()
        return wall, ev0.elapsed_time(ev1) / 1e3


def measure_decode(g, torch, dev, stream, k, n, nbytes, mask, steps, warmup, seed,
                   barrier=None):
    nst = nbytes // (CHUNK * k)
    data = rand_u8(torch, nst * CHUNK * k, seed, dev)
    frags = [torch.empty(nst * CHUNK, dtype=torch.uint8, device=dev) for _ in range(n)]
    L = g.ECMatrixList(k, n)
    sp = stream.cuda_stream
    L.encode_device(dev.index, sp, nst, data, frags)
    rows = g.mask_rows(mask)
    ins = [frags[r - 1] for r in rows]
    out = torch.empty_like(data)
    wall, ev = Timer(torch).run(lambda: L.decode_device(dev.index, sp, nst, mask, ins, out),
                                steps, warmup, barrier)
    ok = bool(torch.equal(out, data))
    return dict(L=L, data=data, frags=frags, out=out, rows=rows, nst=nst, wall=wall,
                kernel_s=ev / steps, ok=ok, user_bytes=nst * CHUNK * k)


def measure_encode(g, torch, dev, stream, k, n, nbytes, steps, warmup, seed):
    nst = nbytes // (CHUNK * k)
    data = rand_u8(torch, nst * CHUNK * k, seed, dev)
    frags = [torch.empty(nst * CHUNK, dtype=torch.uint8, device=dev) for _ in range(n)]
    L = g.ECMatrixList(k, n)
    sp = stream.cuda_stream
    wall, ev = Timer(torch).run(lambda: L.encode_device(dev.index, sp, nst, data, frags),
                                steps, warmup)
    # parity spot check: decode from the last k bricks must return the data
    rows = list(range(n - k + 1, n + 1))
    out = torch.empty_like(data)
    L.decode_device(dev.index, sp, nst, sum(1 << (r - 1) for r in rows),
                    [frags[r - 1] for r in rows], out)
    torch.cuda.synchronize()
    ok = bool(torch.equal(out, data))
    return dict(kernel_s=ev / steps, wall=wall, ok=ok, user_bytes=nst * CHUNK * k)


def gbps(nbytes, seconds):
    return nbytes / seconds / 1e9


def extra_configs(g, torch, dev, stream, steps, warmup):
    ex = {}
    st = max(3, steps // 2)
    # 4+2 encode, 1 GiB
    r = measure_encode(g, torch, dev, stream, 4, 6, 1 << 30, st, warmup, 11)
    ex["enc_4+2_1GiB"] = dict(user_GBps=round(gbps(r["user_bytes"], r["kernel_s"]), 1),
                              hbm_frac=round(gbps(2.5 * r["user_bytes"], r["kernel_s"]) /
                                             HBM_PEAK_GBPS, 4), ok=r["ok"])
    # 8+4, 64K-stripe batches (256 MiB user)
    nb = 65536 * CHUNK * 8
    r = measure_encode(g, torch, dev, stream, 8, 12, nb, st, warmup, 12)
    ex["enc_8+4_64Kstripes"] = dict(user_GBps=round(gbps(r["user_bytes"], r["kernel_s"]), 1),
                                    hbm_frac=round(gbps(2.5 * r["user_bytes"], r["kernel_s"]) /
                                                   HBM_PEAK_GBPS, 4), ok=r["ok"])
    for name, mask in (("dec_8+4_0xFF0", 0xFF0), ("dec_8+4_0xEB5", 0xEB5)):
        r = measure_decode(g, torch, dev, stream, 8, 12, nb, mask, st, warmup, 13)
        ex[name] = dict(user_GBps=round(gbps(r["user_bytes"], r["kernel_s"]), 1),
                        hbm_frac=round(gbps(2 * r["user_bytes"], r["kernel_s"]) /
                                       HBM_PEAK_GBPS, 4), ok=r["ok"])
        del r
    # 4+2 decode, bricks 4 and 5 lost
    r = measure_decode(g, torch, dev, stream, 4, 6, 1 << 30, 0x0F, st, warmup, 14)
    ex["dec_4+2_0x0F"] = dict(user_GBps=round(gbps(r["user_bytes"], r["kernel_s"]), 1),
                              hbm_frac=round(gbps(2 * r["user_bytes"], r["kernel_s"]) /
                                             HBM_PEAK_GBPS, 4), ok=r["ok"])
    del r
    # 16+4 encode, 2 GiB per GPU
    r = measure_encode(g, torch, dev, stream, 16, 20, 2 << 30, st, warmup, 15)
    ex["enc_16+4_2GiB"] = dict(user_GBps=round(gbps(r["user_bytes"], r["kernel_s"]), 1),
                               hbm_frac=round(gbps(2.25 * r["user_bytes"], r["kernel_s"]) /
                                              HBM_PEAK_GBPS, 4), ok=r["ok"])
    torch.cuda.empty_cache()
    return ex


def cpu_baseline(sample_frags, rows, k, budget_s=10.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # test infrastructure: the CPU baseline leg only
    threads = min(16, os.cpu_count() or 1)
    user = sample_frags[0].size * k
    O.decode(k, rows, [f[:CHUNK * 64] for f in sample_frags], nthreads=threads)  # warm
    t0 = time.perf_counter()
    passes = 0
    while True:
        O.decode(k, rows, sample_frags, nthreads=threads)
        passes += 1
        el = time.perf_counter() - t0
        if el >= budget_s or passes >= 2000:
            break
    return dict(value=round(user * passes / el / 1e9, 3), unit="GB/s", cores=threads,
                kind="port",
                sample="oracle/ec_oracle.c decode (ec_code_c_interleaved restatement), 4+2 mask "
                       "0x3C, %d MiB of user data x %d passes, %d threads" %
                       (user >> 20, passes, threads))


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl" if torch.cuda.is_available() else "gloo")
    barrier = (lambda: dist.barrier()) if world > 1 else None
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)
    import glusterfs_amd as g

    k, n, mask = 4, 6, 0x3C
    nbytes = int(args.gib * (1 << 30)) // (CHUNK * k) * (CHUNK * k)
    if args.only:
        # profiling helper (rocprofv3): one config, steps launches, no extras
        k2, n2 = map(int, args.only.split(":")[1].split("+"))
        n2 += k2
        if args.only.startswith("enc"):
            r = measure_encode(g, torch, dev, stream, k2, n2, nbytes, args.steps, args.warmup, 1)
        else:
            m = int(args.only.split(":")[2], 16)
            r = measure_decode(g, torch, dev, stream, k2, n2, nbytes, m, args.steps,
                               args.warmup, 1)
        print(json.dumps(dict(only=args.only, kernel_ms=r["kernel_s"] * 1e3, ok=r["ok"])))
        return

    r = measure_decode(g, torch, dev, stream, k, n, nbytes, mask, args.steps, args.warmup,
                       1234 + rank, barrier)
    wall = r["wall"]
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
        okt = torch.tensor([1 if r["ok"] else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        r["ok"] = bool(okt.item())
    user_total = r["user_bytes"] * world * args.steps
    value = gbps(user_total, wall)
    kernel_s = r["kernel_s"]
    achieved = gbps(2 * r["user_bytes"], kernel_s)

    traffic = None
    tf = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(tf):
        try:
            traffic = json.load(open(tf)).get("dec_4+2_0x3C_1GiB", {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (torch.randint bytes, fixed seed per rank), encoded on-GPU",
        "config": {
            "workload": "disperse 4+2 decode, 2 fragments missing (mask 0x3C), "
                        "%d MiB user data per GPU per step (BASELINE configs[1])" %
                        (r["user_bytes"] >> 20),
            "k": k, "n": n, "mask": "0x3C", "stripes_per_gpu": r["nst"],
            "parallelism": "stripe-range partition, %d GPU(s), no collective" % world,
        },
        "parity_ok": r["ok"],
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic,
            "kernel": "ec_combine<4,false> (decode)",
            "algorithmic_bytes_per_launch": 2 * r["user_bytes"],
            "avg_launch_ms": round(kernel_s * 1e3, 4),
        },
    }
    frags_host = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sample = 128 << 20  # user bytes in the CPU sample
        fs = sample // k
        frags_host = [r["frags"][x - 1][:fs].cpu().numpy() for x in r["rows"]]
    del r
    torch.cuda.empty_cache()
    if not args.no_extra:
        out["extra"] = extra_configs(g, torch, dev, stream, args.steps, args.warmup)
    if frags_host is not None:
        out["cpu_baseline"] = cpu_baseline(frags_host, [3, 4, 5, 6], k)
    if world > 1:
        dist.barrier()
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
