"""GPU parity of host-buffer calls made concurrently from many threads,
the way GlusterFS client threads call the coder (SURVEY.md 8f rank 2:
128 KiB FUSE / write-behind writes up to 4 MiB heal blocks, several volumes
per client, each fop its own call).

Every call runs on its own stream; calls below EC_SPLIT_MIN_MB run whole on
one device (ec_device.hip "device placement").  The tests mix geometries,
masks, buffer kinds and the decode-matrix cache under contention and check
every result bit-exactly against the CPU oracle.  ctypes releases the GIL,
so the Python threads really call the library concurrently.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 512


@pytest.fixture(scope="module")
def ec():
    import glusterfs_amd as g
    if g.device_count() < 1:
        pytest.fail("no MI355X visible: the product has no CPU path")
    return g


def rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


def run_threads(fn, nthreads):
    errs = []

    def wrap(t):
        try:
            fn(t)
        except BaseException as e:  # noqa: BLE001 -- reported below
            errs.append((t, repr(e)))

    th = [threading.Thread(target=wrap, args=(t,)) for t in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


def host_buf(ec, kind, nbytes, keep):
    if kind == "pinned":
        p = ec.PinnedArray(nbytes)
        keep.append(p)
        return p.array
    if kind == "misaligned":
        p = ec.PinnedArray(nbytes + 8)
        keep.append(p)
        return p.array[8:]
    if kind == "pool":            # the integration patch's iobuf memory
        p = ec.PoolBuffer(nbytes)
        keep.append(p)
        return p.array[:nbytes]
    return np.empty(nbytes, np.uint8)


@pytest.mark.parametrize("kind", ["pageable", "pinned", "misaligned", "pool"])
def test_concurrent_mixed_geometries(ec, oracle, kind):
    """16 threads on 4 volumes: encode, decode with a random mask, heal and a
    row-masked encode (a heal write), random sizes from 1 stripe to just
    under the queue limit."""
    geoms = [(4, 6), (8, 12), (16, 20), (5, 7)]
    lists = {g: ec.ECMatrixList(*g) for g in geoms}
    keep = []

    def worker(t):
        rng = np.random.default_rng(100 + t)
        k, n = geoms[t % len(geoms)]
        L = lists[(k, n)]
        for it in range(6):
            nst = int(rng.choice([1, 3, 16, 17, 64, 255, 1000]))
            data = rand_bytes(CHUNK * k * nst, seed=t * 1000 + it)
            src = host_buf(ec, kind, data.size, keep)
            src[:] = data
            frags = [host_buf(ec, kind, CHUNK * nst, keep) for _ in range(n)]
            for f in frags:
                f[:] = 0xA5
            L.encode_batch(nst, src, frags)
            want = oracle.encode(k, n, data)
            for i in range(n):
                assert np.array_equal(frags[i], want[i]), (t, it, "fragment", i)
            rows = sorted(int(r) + 1 for r in rng.choice(n, k, replace=False))
            mask = sum(1 << (r - 1) for r in rows)
            out = host_buf(ec, kind, data.size, keep)
            out[:] = 0
            L.decode_batch(nst, mask, rows, [frags[r - 1] for r in rows], out)
            assert np.array_equal(out, data), (t, it, "decode", hex(mask))
            lost = [b for b in range(n) if not (mask >> b) & 1][:2]
            outs = [host_buf(ec, kind, CHUNK * nst, keep) for _ in lost]
            L.heal(nst, mask, [frags[r - 1] for r in rows], sum(1 << b for b in lost), outs)
            for o, b in zip(outs, lost):
                assert np.array_equal(o, want[b]), (t, it, "heal", b)
            sel = int(rng.integers(1, (1 << n) - 1))
            hw = [host_buf(ec, kind, CHUNK * nst, keep) if (sel >> i) & 1 else None
                  for i in range(n)]
            L.encode_rows(data.size, src, sel, hw)
            for i, o in enumerate(hw):
                if o is not None:
                    assert np.array_equal(o, want[i]), (t, it, "encode_rows", hex(sel), i)

    try:
        run_threads(worker, 16)
    finally:
        for L in lists.values():
            L.fini()
        for p in keep:
            p.free()


def test_many_masks_concurrent_cache(ec, oracle):
    """48 distinct 8+4 masks from 16 threads: the decode-matrix cache
    (ec-method.c:200-256 semantics, max=64) under contention."""
    k, n, nst = 8, 12, 40
    data = [rand_bytes(CHUNK * k * nst, seed=s) for s in range(4)]
    enc = [oracle.encode(k, n, d) for d in data]
    rng = np.random.default_rng(7)
    masks = set()
    while len(masks) < 48:
        masks.add(sum(1 << int(b) for b in rng.choice(n, k, replace=False)))
    masks = sorted(masks)
    with ec.ECMatrixList(k, n, max=64) as L:
        def worker(t):
            for j in range(12):
                m = masks[(t * 12 + j) % len(masks)]
                rows = [b + 1 for b in range(n) if (m >> b) & 1]
                d = (t + j) % 4
                out = np.zeros(CHUNK * k * nst, np.uint8)
                L.decode_batch(nst, m, rows, [enc[d][r - 1] for r in rows], out)
                assert np.array_equal(out, data[d]), (t, j, hex(m))
        run_threads(worker, 16)


def test_drop_in_encode_advances_pointers_under_concurrency(ec, oracle):
    """ec_method_encode (the reference prototype, ec-inode-write.c:2136)
    from 8 threads at the 128 KiB write size, out[] advanced per call."""
    import ctypes
    k, n = 4, 6
    size = 128 << 10
    with ec.ECMatrixList(k, n) as L:
        def worker(t):
            data = rand_bytes(size * 3, seed=500 + t)
            frags = [np.zeros(size * 3 // k, np.uint8) for _ in range(n)]
            arr = (ctypes.c_void_p * n)(*[f.ctypes.data for f in frags])
            for c in range(3):
                ec.ec_method.lib.ec_method_encode(ctypes.byref(L._list), size,
                                       ctypes.c_void_p(data.ctypes.data + c * size), arr)
            for i in range(n):
                assert arr[i] == frags[i].ctypes.data + 3 * size // k
            want = oracle.encode(k, n, data)
            for i in range(n):
                assert np.array_equal(frags[i], want[i]), (t, i)
        run_threads(worker, 8)


def test_device_tables_on_per_thread_streams(ec, oracle):
    """Mixed decodes whose patterns need the device table (> 7 masks of
    16+4), from 8 threads on their per-thread default streams (stream NULL:
    one handle, a different stream per thread), with more distinct mask
    sets than the table cache holds, so entries are evicted while other
    threads' reads may be queued; other threads allocate and free device
    memory meanwhile.  Every output against the oracle."""
    import itertools
    import torch
    k, n, nst, grp = 16, 20, 96, 8
    allm = [sum(1 << b for b in c) for c in itertools.combinations(range(n), k)]
    rng0 = np.random.default_rng(5)
    sets = [sorted(int(x) for x in rng0.choice(allm, 10, replace=False)) for _ in range(40)]
    data = rand_bytes(CHUNK * k * nst, seed=123)
    enc = oracle.encode(k, n, data)
    frags = [torch.from_numpy(f).cuda() for f in enc]
    torch.cuda.synchronize()
    L = ec.ECMatrixList(k, n)

    def worker(t):
        rng = np.random.default_rng(t)
        for it in range(12):
            if t % 4 == 3:            # allocation churn beside the decodes
                x = torch.empty((1 << 20) + int(rng.integers(0, 4096)), dtype=torch.uint8,
                                device="cuda").fill_(t)
                del x
                continue
            masks = sets[int(rng.integers(0, len(sets)))]
            ids = torch.tensor(rng.integers(0, len(masks), nst // grp), dtype=torch.uint8,
                               device="cuda")
            torch.cuda.synchronize()
            out = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
            L.decode_mixed_device(0, None, nst, grp, ids, masks, frags, out)
            ec.sync_device(0)
            assert np.array_equal(out.cpu().numpy(), data), (t, it)

    try:
        run_threads(worker, 8)
    finally:
        L.fini()
