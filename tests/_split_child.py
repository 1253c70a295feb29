"""Child process of tests/test_gpu_split.py (not collected by pytest).

Runs with EC_MI355X_HOST_DEVICES=0,0, EC_MI355X_TEST_SPLIT=1 and
EC_SPLIT_MIN_MB=0, so the library's host-buffer entry points split every call
into two stripe ranges on two "devices" (both GPU 0): the multi-device code of
ec_device.hip partition() -- two host threads, two stages, two streams --
runs on a one-GPU box.  Every output is compared with the oracle bit for bit.
Prints SPLIT-OK on success.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import glusterfs_amd as g  # noqa: E402
import oracle as O         # noqa: E402  (test infrastructure)

CHUNK = 512


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


def main():
    assert g.device_count() >= 1
    # encode_batch, pageable and pinned host buffers, odd stripe counts
    for k, n, nst in ((4, 6, 1001), (16, 20, 333), (5, 7, 257)):
        data = rnd(CHUNK * k * nst, nst)
        want = O.encode(k, n, data)
        with g.ECMatrixList(k, n) as L:
            outs = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n)]
            L.encode_batch(nst, data, outs)
            assert all(np.array_equal(a, b) for a, b in zip(outs, want)), ("enc", k, n)
            pin = [g.PinnedArray(CHUNK * nst) for _ in range(n)]
            with g.PinnedArray(data.size) as pd:
                pd[:] = data
                L.encode_batch(nst, pd, [p.array for p in pin])
            assert all(np.array_equal(p.array, w) for p, w in zip(pin, want)), ("pin", k, n)
            for p in pin:
                p.free()
    # decode_mixed: group boundaries must stay aligned across the split
    for k, n, grp, ng in ((8, 12, 16, 41), (4, 6, 1, 97), (16, 20, 8, 23)):
        nst = grp * ng - (grp > 1)
        frags = [rnd(CHUNK * nst, 50 + f) for f in range(n)]
        rng = np.random.default_rng(k)
        pool = []
        while len(pool) < 9:
            m = sum(1 << int(b) for b in rng.choice(n, k, replace=False))
            if m not in pool:
                pool.append(m)
        masks = [pool[i] for i in rng.integers(0, len(pool), ng)]
        out = np.zeros(CHUNK * k * nst, np.uint8)
        with g.ECMatrixList(k, n) as L:
            L.decode_mixed(nst, grp, masks, frags, out)
        for gi, m in enumerate(masks):
            s0, s1 = gi * grp, min((gi + 1) * grp, nst)
            rows = O.mask_rows(m)
            want = O.decode(k, rows, [frags[r - 1][s0 * CHUNK:s1 * CHUNK] for r in rows])
            assert np.array_equal(out[s0 * CHUNK * k:s1 * CHUNK * k], want), ("mixed", k, gi)
    # heal: regenerate the lost bricks
    for k, n, nst in ((8, 12, 777), (4, 6, 1234)):
        data = rnd(CHUNK * k * nst, 7)
        frags = O.encode(k, n, data)
        good = list(range(n - k, n))
        mask = sum(1 << b for b in good)
        target = ((1 << n) - 1) & ~mask
        outs = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n - k)]
        with g.ECMatrixList(k, n) as L:
            L.heal(nst, mask, [frags[b] for b in good], target, outs)
        assert all(np.array_equal(o, frags[i]) for i, o in enumerate(outs)), ("heal", k)
    print("SPLIT-OK")


if __name__ == "__main__":
    main()
