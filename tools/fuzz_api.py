#!/usr/bin/env python3
"""Differential fuzzer of the drop-in API against the oracle (development
tool, GPU box; runs on the CPU engine too).

For FUZZ_SECS seconds (default 120), FUZZ_THREADS threads (default 8) draw
random calls -- geometry k+r (k 2..16), size (1 stripe .. ~4 MiB), buffer
kind (device tensor, device tensor at an odd byte offset, pinned, registered
range, pool, pageable, misaligned pinned, or a different host kind per
buffer of the call, as a patched client's calls are) and entry
point (encode, encode_rows, decode, decode_mixed, heal, writev_encode, and
the reference's own size-based encode + decode pair; device buffers go
through the _device forms where they differ) -- run
them through glusterfs_amd (ctypes over libec_mi355x.so) and compare every
output byte with the oracle's (oracle/, the test checker).  Buffers of a call
share one kind (mixing host and device is -EINVAL by contract; mixing host
kinds is what the pool / pinned / pageable draws across calls exercise).
Prints a progress line every ~10 s and one JSON summary; exit status 1 on
the first mismatch (its parameters are printed, and FUZZ_SEED replays it).
EC_GPU_ALWAYS=1 keeps host calls on the GPU; FUZZ_KINDS / FUZZ_OPS restrict
the buffer kinds / entry points.  Usage: python tools/fuzz_api.py"""
import json
import mmap
import os
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (torch first: one HIP runtime)
import glusterfs_amd as g  # noqa: E402
import oracle as O  # noqa: E402  (the checker)

CHUNK = 512
GEOS = [(2, 1), (3, 2), (4, 2), (5, 2), (6, 3), (8, 4), (8, 3), (10, 4), (12, 4), (16, 4), (16, 8)]
OPS = ["encode", "encode_rows", "decode", "decode_mixed", "heal", "writev", "dropin", "volume",
       "stream_chain"]


class Arena:
    """Buffers of one kind for one call; freed together."""

    def __init__(self, kind, dev, rng=None):
        self.kind, self.dev, self.keep, self.regs, self.keep_raw = kind, dev, [], [], []
        self.keep_dev = []
        self.rng = rng or random.Random(0)
        self.subs = []

    def buf(self, data=None, nbytes=None):
        if self.kind == "mixed_host":   # every buffer of the call its own host kind
            sub = Arena(self.rng.choice(["pinned", "registered", "pool", "pageable", "misaligned"]),
                        self.dev)
            self.subs.append(sub)
            return sub.buf(data, nbytes)
        n = data.size if data is not None else nbytes
        if self.kind in ("device", "device_offset"):
            off = 3 if self.kind == "device_offset" else 0   # a tensor slice at an odd byte
            t = torch.empty(n + off, dtype=torch.uint8, device=self.dev)[off:]
            if data is not None:
                t.copy_(torch.from_numpy(data))
            # held until the call has synchronised (free()): a device call is
            # asynchronous on the caller's per-thread stream, which torch's
            # allocator does not track, so a tensor passed as a temporary
            # would go back to the allocator -- and to another thread's
            # buffer -- while the library's kernels may still read it (r04af
            # passed the partial write's user buffer that way)
            self.keep_dev.append(t)
            return t
        if self.kind == "registered":     # an existing mapping registered (an iobuf arena)
            m = mmap.mmap(-1, (n + 4095) // 4096 * 4096)
            a = np.frombuffer(m, np.uint8)
            rc = g.ec_method.lib.ec_method_host_register(a.ctypes.data, a.nbytes)
            if rc == 0:
                self.regs.append(a.ctypes.data)
            self.keep_raw.append(m)
            a = a[:n]
            if data is not None:
                a[:] = data
            return a
        if self.kind in ("pinned", "misaligned"):  # noqa: SIM114
            extra = 8 if self.kind == "misaligned" else 0
            p = g.PinnedArray(n + extra)
            self.keep.append(p)
            a = p.array[extra:extra + n]
        elif self.kind == "pool":
            p = g.PoolBuffer(n)
            self.keep.append(p)
            a = p.array[:n]
        else:
            a = np.empty(n, np.uint8)
        if data is not None:
            a[:] = data
        return a

    def free(self):
        for sub in self.subs:
            sub.free()
        for p in self.keep:
            p.free()
        for p in self.regs:
            g.ec_method.lib.ec_method_host_unregister(p)
        self.keep_dev.clear()


def host(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


def same(desc, name, got, want):
    """Byte equality; on a difference, note where in desc (first offset,
    count, and whether the buffer holds the oracle's bytes elsewhere)."""
    got = host(got)
    if np.array_equal(got, want):
        return True
    d = np.nonzero(got != want)[0]
    desc.setdefault("diff", []).append(dict(buf=name, first=int(d[0]), count=int(d.size),
                                            size=int(want.size), zeros=bool((got == 0).all())))
    return False


def one_call(rng, lists, dev):
    k, r = rng.choice(GEOS)
    n = k + r
    L = lists[(k, r)]
    ops = [o for o in OPS if o in os.environ.get("FUZZ_OPS", "").split()] or OPS
    op = rng.choice(ops)
    if op == "stream_chain" and dev is None:
        op = "encode"                          # device-resident only
    kinds = ["device", "device_offset", "pinned", "registered", "pool", "pageable",
             "misaligned", "mixed_host"] if dev is not None else ["pool", "pageable"]
    only = os.environ.get("FUZZ_KINDS")          # e.g. "device_offset registered"
    if only:
        kinds = [x for x in kinds if x in only.split()] or kinds
    kind = rng.choice(kinds)

    nst = rng.choice([1, 2, 7, 8, 9, 31, 64, 100, 257, 1000, 1031,
                      max(1, (4 << 20) // (CHUNK * k))])
    seed = rng.randrange(1 << 30)
    drng = np.random.default_rng(seed)
    data = drng.integers(0, 256, CHUNK * k * nst, dtype=np.uint8)
    desc = dict(op=op, k=k, n=n, kind=kind, nst=nst, seed=seed)
    A = Arena(kind, dev, rng)
    try:
        if op == "encode":
            src = A.buf(data)
            outs = [A.buf(nbytes=CHUNK * nst) for _ in range(n)]
            L.encode_batch(nst, src, outs)
            want = O.encode(k, n, data)
            return desc, all([same(desc, "frag%d" % i, o, w) for i, (o, w) in enumerate(zip(outs, want))])
        if op == "stream_chain":
            if not kind.startswith("device"):
                kind = desc["kind"] = "device"
                A.kind = "device"
            # device-resident calls queued on a side stream with no sync in
            # between (stream order is the only ordering): encode, a mixed
            # decode over up to 40 masks (past the kernel-argument segment:
            # the device pattern table and its per-stream cache), a heal
            src = A.buf(data)
            frags = [A.buf(nbytes=CHUNK * nst) for _ in range(n)]
            grp = rng.choice([8, 16, 64])
            ng = (nst + grp - 1) // grp
            pool = []
            for _ in range(rng.randint(1, 40)):
                pool.append(sum(1 << (x - 1) for x in sorted(rng.sample(range(1, n + 1), k))))
            uniq = sorted(set(pool))
            ids = torch.tensor([rng.randrange(len(uniq)) for _ in range(ng)], dtype=torch.uint8,
                               device=dev)
            out = A.buf(nbytes=data.size)
            rows = sorted(rng.sample(range(1, n + 1), k))
            m = sum(1 << (x - 1) for x in rows)
            lost = [b for b in range(n) if not (m >> b) & 1]
            tgt = sorted(rng.sample(lost, rng.randint(1, len(lost))))
            houts = [A.buf(nbytes=CHUNK * nst) for _ in tgt]
            desc.update(masks=len(uniq), grp=grp, mask=m)
            st = torch.cuda.Stream(device=dev)
            st.wait_stream(torch.cuda.current_stream(dev))
            L.encode_device(dev.index, st.cuda_stream, nst, src, frags)
            L.decode_mixed_device(dev.index, st.cuda_stream, nst, grp, ids, uniq, frags, out)
            L.heal_device(dev.index, st.cuda_stream, nst, m, [frags[x - 1] for x in rows],
                          sum(1 << b for b in tgt), houts)
            st.synchronize()
            want = O.encode(k, n, data)
            return desc, all([same(desc, "frag%d" % i, f, w) for i, (f, w) in enumerate(zip(frags, want))]) \
                and same(desc, "decoded", out, data) and \
                all([same(desc, "heal%d" % b, h, want[b]) for h, b in zip(houts, tgt)])
        if op == "volume":
            # a volume brought up and torn down while others code (ec.c:837
            # init, :198 fini), with a random cpu-extensions value
            gen = rng.choice(["auto", "hip"] if kind.startswith("device") else
                             ["auto", "none", "avx", "x64", "hip"])
            desc["gen"] = gen
            src = A.buf(data)
            outs = [A.buf(nbytes=CHUNK * nst) for _ in range(n)]
            with g.ECMatrixList(k, n, gen=gen) as V:
                V.encode_batch(nst, src, outs)
                rows = sorted(rng.sample(range(1, n + 1), k))
                m = sum(1 << (x - 1) for x in rows)
                desc["mask"] = m
                out = A.buf(nbytes=data.size)
                V.decode_batch(nst, m, rows, [outs[x - 1] for x in rows], out)
            want = O.encode(k, n, data)
            return desc, all([same(desc, "frag%d" % i, o, w)
                              for i, (o, w) in enumerate(zip(outs, want))]) and \
                same(desc, "decoded", out, data)
        if op == "dropin":
            # the reference's own two calls (ec-method.h:31-46): encode by
            # size, then decode by fragment size from a random brick set
            src = A.buf(data)
            outs = [A.buf(nbytes=CHUNK * nst) for _ in range(n)]
            L.encode(data.size, src, outs)
            rows = sorted(rng.sample(range(1, n + 1), k))
            m = sum(1 << (x - 1) for x in rows)
            desc["mask"] = m
            out = A.buf(nbytes=data.size)
            want = O.encode(k, n, data)
            enc_ok = all([same(desc, "frag%d" % i, o, w) for i, (o, w) in enumerate(zip(outs, want))])
            L.decode(CHUNK * nst, m, rows, [outs[x - 1] for x in rows], out)
            return desc, same(desc, "decoded", out, data) and enc_ok
        if op == "encode_rows":
            m = rng.randrange(1, 1 << n)
            desc["mask"] = m
            src = A.buf(data)
            outs = [A.buf(nbytes=CHUNK * nst) if (m >> i) & 1 else None for i in range(n)]
            if kind.startswith("device"):
                L.encode_rows_device(dev.index, None, nst, src, m, outs)
                g.sync_device(dev.index)
            else:
                L.encode_rows(data.size, src, m, outs)
            want = O.encode(k, n, data)
            return desc, all([same(desc, "frag%d" % i, o, want[i]) for i, o in enumerate(outs)
                              if o is not None])
        frags_np = [drng.integers(0, 256, CHUNK * nst, dtype=np.uint8) for _ in range(n)]
        rows = sorted(rng.sample(range(1, n + 1), k))
        mask = sum(1 << (x - 1) for x in rows)
        desc["mask"] = mask
        if op == "decode":
            fr = [A.buf(frags_np[x - 1]) for x in rows]
            out = A.buf(nbytes=CHUNK * k * nst)
            L.decode_batch(nst, mask, rows, fr, out)
            return desc, same(desc, "decoded", out, O.decode(k, rows, [frags_np[x - 1]
                                                                         for x in rows]))
        if op == "heal":
            fr = [A.buf(frags_np[x - 1]) for x in rows]
            lost = [b for b in range(n) if not (mask >> b) & 1]
            tgt = rng.sample(lost, rng.randint(1, len(lost)))
            tmask = sum(1 << b for b in tgt)
            outs = [A.buf(nbytes=CHUNK * nst) for _ in tgt]
            L.heal(nst, mask, fr, tmask, outs)
            full = O.encode(k, n, O.decode(k, rows, [frags_np[x - 1] for x in rows]))
            return desc, all([same(desc, "frag%d" % b, o, full[b])
                              for o, b in zip(outs, sorted(tgt))])
        if op == "decode_mixed":
            grp = rng.choice([1, 2, 4, 8, 16, 64])
            ng = (nst + grp - 1) // grp
            pool_masks = [mask] + [sum(1 << (x - 1) for x in sorted(rng.sample(range(1, n + 1), k)))
                                   for _ in range(rng.randint(0, 5))]
            gm = [rng.choice(pool_masks) for _ in range(ng)]
            fr = [A.buf(f) for f in frags_np]
            out = A.buf(nbytes=CHUNK * k * nst)
            if kind.startswith("device"):
                uniq = sorted(set(gm))
                ids = torch.tensor([uniq.index(x) for x in gm], dtype=torch.uint8, device=dev)
                L.decode_mixed_device(dev.index, None, nst, grp, ids, uniq, fr, out)
                g.sync_device(dev.index)
            else:
                L.decode_mixed(nst, grp, gm, fr, out)
            got = host(out)
            for gi, m in enumerate(gm):
                a0, a1 = gi * grp * CHUNK, min(nst, (gi + 1) * grp) * CHUNK
                rw = O.mask_rows(m)
                exp = O.decode(k, rw, [frags_np[x - 1][a0:a1] for x in rw])
                if not np.array_equal(got[a0 * k:a1 * k], exp):
                    return desc, False
            return desc, True
        # writev: a partial-stripe write at a random head with old stripes
        S = CHUNK * k
        head = rng.randrange(S)
        us = rng.randrange(1, max(2, CHUNK * k * nst - head))
        user = data[:us]
        oh = drng.integers(0, 256, S, dtype=np.uint8) if rng.random() < 0.7 else None
        ot = drng.integers(0, 256, S, dtype=np.uint8) if rng.random() < 0.7 else None
        desc.update(head=head, user=us)
        size = (head + us + S - 1) // S * S
        outs = [A.buf(nbytes=size // k) for _ in range(n)]
        if kind.startswith("device"):
            L.writev_encode_device(dev.index, None, head, us, A.buf(user),
                                   None if oh is None else A.buf(oh),
                                   None if ot is None else A.buf(ot), outs)
            g.sync_device(dev.index)
        else:
            L.writev_encode(head, A.buf(user), None if oh is None else A.buf(oh),
                            None if ot is None else A.buf(ot), outs)
        want = O.encode(k, n, O.writev_merge(k, head, user, oh, ot))
        return desc, all([same(desc, "frag%d" % i, o, w) for i, (o, w) in enumerate(zip(outs, want))])
    finally:
        A.free()


def main():
    secs = float(os.environ.get("FUZZ_SECS", "120"))
    nth = int(os.environ.get("FUZZ_THREADS", "8"))
    seed0 = int(os.environ.get("FUZZ_SEED", str(int(time.time()))))
    dev = torch.device("cuda:0") if g.device_count() > 0 else None
    lists = {gk: g.ECMatrixList(gk[0], gk[0] + gk[1]) for gk in GEOS}
    counts = {op: 0 for op in OPS}
    bad = []
    lock = threading.Lock()
    t_end = time.time() + secs

    def worker(t):
        rng = random.Random(seed0 * 1000 + t)
        while time.time() < t_end and not bad:
            try:
                desc, ok = one_call(rng, lists, dev)
            except Exception as e:  # noqa: BLE001 -- any error is a finding
                desc, ok = dict(error=repr(e)[:300]), False
            with lock:
                if ok:
                    counts[desc["op"]] += 1
                else:
                    bad.append(desc)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(nth)]
    for t in th:
        t.start()
    last = time.time()
    while any(t.is_alive() for t in th):
        time.sleep(0.5)
        if time.time() - last >= 10:
            last = time.time()
            print("fuzz: %d calls, %d bad" % (sum(counts.values()), len(bad)), flush=True)
    for t in th:
        t.join()
    st = g.ec_method.stats()
    for L in lists.values():
        L.fini()
    print(json.dumps(dict(seed=seed0, threads=nth, secs=secs, calls=counts,
                          gpu_calls=st["gpu_calls"], cpu_calls=st["cpu_calls"],
                          cpu_fallbacks=st["cpu_fallbacks"], jit=g.jit_stats(),
                          mismatches=bad[:5])), flush=True)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
