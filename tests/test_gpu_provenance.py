"""GPU parity of the buffer provenances a patched GlusterFS client hands the
coder (VERDICT r03 missing #1 and #3):

* the pinned buffer pool (ec_method_buffer_get / _put) that the patch's iobuf
  data allocator uses for every non-arena iobuf -- iobuf_get_from_small
  (<= 128 KiB) and iobuf_get_from_stdalloc (> 1 MiB), iobuf.c:439-510, i.e.
  every ec_buffer_alloc size class outside the arenas (ec-helpers.c:134-165);
* iobuf arenas registered by the deferred registration thread
  (ec_method_host_register_async: the arena hook runs under
  iobuf_pool->mutex, iobuf.c:157);
* calls that mix them with pageable buffers, buffer by buffer: RPC reply
  fragments (ec-inode-read.c:1173-1176) in a registered arena and the output
  in plain malloc memory, or the reverse (the device layer reads mapped
  buffers in place and stages only the others).

Every result is compared with the CPU oracle.  conftest.py sets
EC_GPU_ALWAYS=1, so every call here runs on the GPU."""
import ctypes
import mmap

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


class Arena:
    """An iobuf arena: one anonymous mapping (iobuf.c:151-157), registered
    through the deferred queue like the patch's arena hook does, carved into
    equal pages."""

    def __init__(self, ec, page, count, flush=True):
        self.ec, self.page, self.size = ec, page, page * count
        self.m = mmap.mmap(-1, self.size)
        self.a = np.frombuffer(self.m, np.uint8)
        self.ptr = self.a.ctypes.data
        assert ec.ec_method.lib.ec_method_host_register_async(self.ptr, self.size) == 0
        if flush:
            ec.ec_method.lib.ec_method_host_register_flush()

    def pages(self):
        return [self.a[i * self.page:(i + 1) * self.page] for i in range(self.size // self.page)]

    def close(self):
        assert self.ec.ec_method.lib.ec_method_host_unregister(self.ptr) == 0
        self.a = None
        try:
            self.m.close()
        except BufferError:       # views still alive: unmapped when collected
            pass


def test_pool_buffers_classes_and_recycling(ec):
    """Every size class ec_buffer_alloc produces outside the arenas: small
    iobufs (<= 128 KiB + 64), heal-window outputs (4 MiB + 64 + 4095 of
    stdalloc alignment slack, 6 MiB + 64 + 4095), and the 128 MiB limit."""
    lib = ec.ec_method.lib
    sizes = [4096, 5000, 32 << 10, (128 << 10), (1 << 20), (1 << 20) + 1, (4 << 20) + 64 + 4095,
             (6 << 20) + 64 + 4095, 128 << 20]
    st0 = ec.pool_stats()
    bufs = [lib.ec_method_buffer_get(s) for s in sizes]
    assert all(bufs), bufs
    assert all(b % 4096 == 0 for b in bufs)
    spans = sorted((b, b + s) for b, s in zip(bufs, sizes))
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])), "overlapping pool buffers"
    assert not lib.ec_method_buffer_get((128 << 20) + 1)           # past the largest run
    for b, s in zip(bufs, sizes):                                  # writable end to end
        ctypes.memset(b, 0x5A, s)
    for b in bufs:
        assert lib.ec_method_buffer_put(b) == 1
    again = [lib.ec_method_buffer_get(s) for s in sizes]
    assert sorted(again) == sorted(bufs), "freed buffers are not reused"
    for b in again:
        assert lib.ec_method_buffer_put(b) == 1
    a = np.empty(4096, np.uint8)
    assert lib.ec_method_buffer_put(a.ctypes.data) == 0            # not the pool's
    assert lib.ec_method_buffer_put(bufs[0] + 64) == 0             # inside, not a buffer
    st1 = ec.pool_stats()
    assert st1["gets"] - st0["gets"] == 2 * len(sizes) + 1
    assert st1["misses"] - st0["misses"] == 1                     # the 128 MiB + 1 request
    assert st1["in_use_bytes"] == st0["in_use_bytes"]
    assert st1["slabs"] >= 1 and st1["pool_bytes"] >= (128 << 20)


@pytest.mark.parametrize("k,n", [(4, 6), (8, 12), (16, 20)])
def test_heal_window_in_pool_buffers(ec, oracle, k, n):
    """A self-heal window as a patched glustershd codes it: fragments in
    registered 1 MiB-page arenas (RPC replies, iobuf.c:25-26), decode output
    and re-encode output from ec_buffer_alloc -> stdalloc -> the pool."""
    W = 4 << 20
    nst = W // (CHUNK * k)
    fl = nst * CHUNK
    data = rand_bytes(W, seed=k)
    enc = oracle.encode(k, n, data)
    page = 1 << 20
    per = max(1, page // fl)
    arenas = [Arena(ec, page, 2) for _ in range((n + 2 * per - 1) // (2 * per))]
    pages = [p for a in arenas for p in a.pages()]
    frags = []
    for i in range(n):
        pg = pages[i // per]
        f = pg[(i % per) * fl:(i % per + 1) * fl]
        f[:] = enc[i]
        frags.append(f)
    dec = ec.PoolBuffer(W + 64 + 4095)
    reenc = ec.PoolBuffer(n * fl + 64 + 4095)
    try:
        assert dec.pooled and reenc.pooled
        out = dec.array[:W]
        rows = list(range(n - k + 1, n + 1))
        mask = sum(1 << (r - 1) for r in rows)
        st0 = ec.stats()
        with ec.ECMatrixList(k, n) as L:
            L.decode(fl, mask, rows, [frags[r - 1] for r in rows], out)
            assert np.array_equal(out, data)
            outs = [reenc.array[i * fl:(i + 1) * fl] for i in range(n)]
            L.encode(W, out, outs)
            for i in range(n):
                assert np.array_equal(outs[i], enc[i]), i
        assert ec.stats()["gpu_calls"] - st0["gpu_calls"] == 2
    finally:
        dec.free()
        reenc.free()
        for a in arenas:
            a.close()


@pytest.mark.parametrize("which", ["frags_mapped", "out_mapped"])
@pytest.mark.parametrize("k,n", [(4, 6), (8, 12), (16, 20)])
def test_mixed_provenance_decode_encode_heal(ec, oracle, which, k, n):
    """One call, two provenances.  frags_mapped: registered-arena fragments
    (RPC replies) with a pageable decode output, then an encode of that
    pageable buffer into pool outputs, and a heal into pool outputs.
    out_mapped: the reverse -- pageable fragments, pool output, encode of the
    pool buffer into pageable outputs, heal into pageable outputs."""
    nst = 3 * 1024 + 5                      # several zero-copy tiles, ragged
    fl = nst * CHUNK
    data = rand_bytes(fl * k, seed=100 + k)
    enc = oracle.encode(k, n, data)
    arena = Arena(ec, fl, n)
    pool = []

    def pooled(nbytes):
        b = ec.PoolBuffer(nbytes)
        assert b.pooled
        pool.append(b)
        return b.array

    def other(nbytes):
        """the provenance opposite to the call's input"""
        return pooled(nbytes) if which == "frags_mapped" else np.zeros(nbytes, np.uint8)

    try:
        if which == "frags_mapped":
            frags = arena.pages()
            for i in range(n):
                frags[i][:] = enc[i]
        else:
            frags = [np.array(e) for e in enc]
        out = np.zeros(fl * k, np.uint8) if which == "frags_mapped" else pooled(fl * k)
        rows = sorted(int(r) + 1 for r in np.random.default_rng(k).choice(n, k, replace=False))
        mask = sum(1 << (r - 1) for r in rows)
        with ec.ECMatrixList(k, n) as L:
            L.decode(fl, mask, rows, [frags[r - 1] for r in rows], out)
            assert np.array_equal(out, data)
            eouts = [other(fl) for _ in range(n)]
            L.encode(fl * k, out, eouts)
            for i in range(n):
                assert np.array_equal(eouts[i], enc[i]), ("enc", i)
            lost = [b for b in range(n) if not (mask >> b) & 1][:2]
            tmask = sum(1 << b for b in lost)
            hout = [other(fl) for _ in lost]
            L.heal(nst, mask, [frags[r - 1] for r in rows], tmask, hout)
            for j, b in enumerate(lost):
                assert np.array_equal(hout[j], enc[b]), ("heal", b)
    finally:
        for b in pool:
            b.free()
        arena.close()


def test_deferred_registration_queue(ec, oracle):
    """Ranges queued for registration are coded correctly before and after
    the library thread registers them; unregistering a queued range drops it
    (the arena hook may unmap an arena right after adding it)."""
    lib = ec.ec_method.lib
    st0 = ec.pool_stats()
    # queued, then dropped before the thread gets to most of them
    maps = [mmap.mmap(-1, 2 << 20) for _ in range(16)]
    ptrs = [np.frombuffer(m, np.uint8).ctypes.data for m in maps]
    for p in ptrs:
        assert lib.ec_method_host_register_async(p, 2 << 20) == 0
    for p in ptrs:
        assert lib.ec_method_host_unregister(p) == 0
    lib.ec_method_host_register_flush()
    del ptrs
    for m in maps:
        m.close()
    # coded while (possibly) still queued, then after registration
    k, n, nst = 8, 12, 2048
    fl = nst * CHUNK
    data = rand_bytes(fl * k, seed=77)
    enc = oracle.encode(k, n, data)
    arena = Arena(ec, fl, n, flush=False)
    try:
        frags = arena.pages()
        for i in range(n):
            frags[i][:] = enc[i]
        out = np.zeros(fl * k, np.uint8)
        rows = list(range(5, 13))
        with ec.ECMatrixList(k, n) as L:
            L.decode(fl, 0xFF0, rows, [frags[r - 1] for r in rows], out)
            assert np.array_equal(out, data)
            lib.ec_method_host_register_flush()
            out[:] = 0
            L.decode(fl, 0xFF0, rows, [frags[r - 1] for r in rows], out)
            assert np.array_equal(out, data)
    finally:
        arena.close()
    st1 = ec.pool_stats()
    assert st1["deferred_registers"] > st0["deferred_registers"]
    assert st1["deferred_register_failures"] == st0["deferred_register_failures"]
    assert st1["unregisters"] >= st0["unregisters"] + 1


def test_pool_concurrent_get_put(ec):
    """Eight threads take and return pool buffers of mixed size classes
    (small slabs and granule runs) at once, each filling its buffer with its
    own tag and checking it before the put: no buffer is ever handed to two
    holders, and every get is matched by its put."""
    import threading
    lib = ec.ec_method.lib
    sizes = [4096, 9000, 64 << 10, 200 << 10, 1 << 20, (2 << 20) + 5, (4 << 20) + 4159]
    st0 = ec.pool_stats()
    errors = []

    def worker(tag):
        rng = np.random.default_rng(tag)
        held = []
        try:
            for it in range(300):
                if held and (len(held) > 6 or rng.random() < 0.5):
                    p, n = held.pop(int(rng.integers(len(held))))
                    a = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p))
                    if not (a[0] == tag and a[n - 1] == tag and a[n // 2] == tag):
                        errors.append("buffer %#x of thread %d overwritten" % (p, tag))
                    if lib.ec_method_buffer_put(p) != 1:
                        errors.append("put refused %#x" % p)
                else:
                    n = sizes[int(rng.integers(len(sizes)))]
                    p = lib.ec_method_buffer_get(n)
                    if not p:
                        errors.append("get(%d) failed" % n)
                        continue
                    ctypes.memset(p, tag, n)
                    held.append((p, n))
        finally:
            for p, n in held:
                lib.ec_method_buffer_put(p)

    th = [threading.Thread(target=worker, args=(t + 1,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    st1 = ec.pool_stats()
    assert st1["in_use_bytes"] == st0["in_use_bytes"]
    assert st1["misses"] == st0["misses"]
