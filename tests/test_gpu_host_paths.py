"""GPU parity of the host-buffer paths (ec_device.hip "host-buffer pipeline").

Host buffers are either coded in place over PCIe (pinned, device-mapped,
16-byte aligned) or staged through pinned slots by CPU threads (pageable or
misaligned); one call may mix both kinds.  Sizes span several pipeline
batches (32 MiB staged, 256 MiB in place) so slot rotation and ragged final
batches are exercised.  Bit-exact against the CPU oracle.
"""
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


class Bufs:
    """Allocates host buffers of one kind: 'pinned', 'pageable',
    'misaligned' (pinned + 8 bytes: must fall back to staging) or
    'registered' (pageable pinned through ec_method_host_register)."""

    def __init__(self, ec, kind):
        self.ec, self.kind, self.keep, self.regs, self.maps = ec, kind, [], [], []

    def new(self, nbytes, fill=None):
        if self.kind == "pageable":
            a = np.empty(nbytes, np.uint8)
        elif self.kind == "registered":
            # its own page-aligned mapping, as an iobuf arena: registrations
            # that share a page are refused (ec_device.hip RangeSet)
            import mmap
            m = mmap.mmap(-1, (nbytes + 4095) // 4096 * 4096)
            a = np.frombuffer(m, np.uint8)[:nbytes]
            r = self.ec.host_registered(a)
            r.__enter__()
            self.regs.append(r)
            self.maps.append((m, a))
        else:
            extra = 8 if self.kind == "misaligned" else 0
            p = self.ec.PinnedArray(nbytes + extra)
            self.keep.append(p)
            a = p.array[extra:]
        if fill is not None:
            a[:] = fill
        return a

    def close(self):
        for r in self.regs:
            r.__exit__()
        for p in self.keep:
            p.free()
        self.regs, self.maps = [], []     # the mappings go with their last views


KINDS = ["pinned", "pageable", "misaligned", "registered", "mixed"]


def _alloc(ec, kind, i):
    """kind 'mixed' alternates pinned / pageable per buffer."""
    if kind == "mixed":
        return "pinned" if i % 2 == 0 else "pageable"
    return kind


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("k,n", [(4, 6), (8, 12), (5, 7), (10, 13), (16, 20)])
def test_encode_decode_host_kinds(ec, oracle, kind, k, n):
    # 2-3 staged batches with a ragged tail; k + rows up to 32 exercises the
    # 128 KiB-LDS zero-copy combine (10+3: generic encode, 16+4: decode)
    nst = 40000 if k <= 5 else 20000 if k <= 8 else 9000
    data = rand_bytes(CHUNK * k * nst, seed=k * 7 + n)
    want = oracle.encode(k, n, data, nthreads=8)
    pools = {t: Bufs(ec, t) for t in ("pinned", "pageable", "misaligned", "registered")}
    try:
        src = pools[_alloc(ec, kind, 0)].new(data.size, data)
        frags = [pools[_alloc(ec, kind, i + 1)].new(CHUNK * nst, 0xA5) for i in range(n)]
        rows = sorted(int(r) + 1 for r in np.random.default_rng(k).choice(n, k, replace=False))
        mask = sum(1 << (r - 1) for r in rows)
        out = pools[_alloc(ec, kind, 1)].new(data.size, 0)
        with ec.ECMatrixList(k, n) as L:
            L.encode_batch(nst, src, frags)
            for i in range(n):
                assert np.array_equal(frags[i], want[i]), "fragment %d" % i
            L.decode_batch(nst, mask, rows, [frags[r - 1] for r in rows], out)
        assert np.array_equal(out, data)
    finally:
        for p in pools.values():
            p.close()


def test_in_place_multi_batch(ec, oracle):
    """All-pinned 4+2 over more than one in-place batch (256 MiB input)."""
    k, n = 4, 6
    nst = (300 << 20) // (CHUNK * k)
    pool = Bufs(ec, "pinned")
    try:
        src = pool.new(CHUNK * k * nst)
        src[:] = rand_bytes(src.size, seed=5)
        frags = [pool.new(CHUNK * nst) for _ in range(n)]
        out = pool.new(src.size, 0)
        with ec.ECMatrixList(k, n) as L:
            L.encode_batch(nst, src, frags)
            want = oracle.encode(k, n, src[:CHUNK * k * 4096], nthreads=8)
            for i in range(n):                   # prefix vs oracle ...
                assert np.array_equal(frags[i][:CHUNK * 4096], want[i])
            rows = [3, 4, 5, 6]                  # ... whole range by round trip
            L.decode_batch(nst, 0x3C, rows, [frags[r - 1] for r in rows], out)
        assert np.array_equal(out, src)
    finally:
        pool.close()


@pytest.mark.parametrize("kind", ["pinned", "pageable", "mixed"])
def test_decode_mixed_and_heal_host_kinds(ec, oracle, kind):
    k, n, group = 4, 6, 64
    nst = 100000 - 17                          # several batches, ragged last group
    data = rand_bytes(CHUNK * k * nst, seed=9)
    enc = oracle.encode(k, n, data, nthreads=8)
    pools = {t: Bufs(ec, t) for t in ("pinned", "pageable")}
    try:
        frags = [pools[_alloc(ec, kind, i)].new(CHUNK * nst, enc[i]) for i in range(n)]
        out = pools[_alloc(ec, kind, 1)].new(data.size, 0)
        ngroups = (nst + group - 1) // group
        rng = np.random.default_rng(2)
        pool_masks = [0x3C, 0x0F, 0x33, 0x2B]
        masks = [pool_masks[i] for i in rng.integers(0, len(pool_masks), ngroups)]
        with ec.ECMatrixList(k, n) as L:
            L.decode_mixed(nst, group, masks, frags, out)
            assert np.array_equal(out, data)
            outs = [pools[_alloc(ec, kind, i)].new(CHUNK * nst, 0) for i in range(2)]
            rows = [3, 4, 5, 6]
            L.heal(nst, 0x3C, [frags[r - 1] for r in rows], 0x03, outs)
            assert np.array_equal(outs[0], enc[0]) and np.array_equal(outs[1], enc[1])
    finally:
        for p in pools.values():
            p.close()


@pytest.mark.parametrize("kind", ["pinned", "pageable"])
def test_decode_mixed_small_groups_host_kinds(ec, oracle, kind):
    """2-stripe pattern groups through the host-buffer pipeline (zero-copy
    for pinned, staged for pageable), several batches."""
    k, n, group = 4, 6, 2
    nst = 40000 - 1
    data = rand_bytes(CHUNK * k * nst, seed=19)
    enc = oracle.encode(k, n, data, nthreads=8)
    p = Bufs(ec, kind)
    try:
        frags = [p.new(CHUNK * nst, enc[i]) for i in range(n)]
        out = p.new(data.size, 0)
        ngroups = (nst + group - 1) // group
        rng = np.random.default_rng(3)
        pool_masks = [0x3C, 0x0F, 0x33, 0x2B, 0x1E]
        masks = [pool_masks[i] for i in rng.integers(0, len(pool_masks), ngroups)]
        with ec.ECMatrixList(k, n) as L:
            L.decode_mixed(nst, group, masks, frags, out)
        assert np.array_equal(out, data)
    finally:
        p.close()


@pytest.mark.parametrize("kind", ["pinned", "pageable"])
@pytest.mark.parametrize("group", [8, 16])
def test_decode_16p4_host_kinds(ec, oracle, kind, group):
    """16+4 decodes of host buffers: the 16-row combine runs the persistent
    zero-copy kernel on 4-stripe tiles (two 8-stripe input tiles and the
    output tile would not fit the CU's LDS), single-pattern and mixed with
    8- and 16-stripe pattern groups, ragged ends."""
    k, n = 16, 20
    nst = 3 * 1024 + 13           # >= 2048 stripes: the 4-stripe persistent kernel
    data = rand_bytes(CHUNK * k * nst, seed=group + 31)
    enc = oracle.encode(k, n, data, nthreads=8)
    p = Bufs(ec, kind)
    try:
        frags = [p.new(CHUNK * nst, enc[i]) for i in range(n)]
        out = p.new(data.size, 0)
        rng = np.random.default_rng(group)
        pool_masks = [0xFFFF0, 0x0FFFF, 0xF0FFF, 0xFF0FF, 0x7FFF8]
        ngroups = (nst + group - 1) // group
        masks = [pool_masks[i] for i in rng.integers(0, len(pool_masks), ngroups)]
        s0 = ec.ec_method.stats()
        with ec.ECMatrixList(k, n) as L:
            for m in pool_masks[:2]:
                rows = [b + 1 for b in range(n) if (m >> b) & 1]
                out[:] = 0
                L.decode_batch(nst, m, rows, [frags[r - 1] for r in rows], out)
                assert np.array_equal(out, data), hex(m)
            out[:] = 0
            L.decode_mixed(nst, group, masks, frags, out)
            assert np.array_equal(out, data)
        assert ec.ec_method.stats()["cpu_fallbacks"] == s0["cpu_fallbacks"]
    finally:
        p.close()


@pytest.mark.parametrize("kind", ["pinned", "pageable"])
@pytest.mark.parametrize("nst", [2047, 3 * 1024 + 13])
def test_encode_16p4_host_kinds(ec, oracle, kind, nst):
    """16+4 encodes of host buffers (r06): from 2048 stripes the encode runs
    as a combine with the encode matrix as its pattern (20 rows of the
    4-stripe double-buffered zero-copy kernel), below it the register
    encoder; every fragment against the oracle, no CPU fallback."""
    k, n = 16, 20
    data = rand_bytes(CHUNK * k * nst, seed=nst)
    want = oracle.encode(k, n, data, nthreads=8)
    p = Bufs(ec, kind)
    try:
        src = p.new(data.size, data)
        frags = [p.new(CHUNK * nst, 0) for _ in range(n)]
        s0 = ec.ec_method.stats()
        with ec.ECMatrixList(k, n) as L:
            L.encode_batch(nst, src, frags)
        for i in range(n):
            assert np.array_equal(frags[i], want[i]), i
        assert ec.ec_method.stats()["cpu_fallbacks"] == s0["cpu_fallbacks"]
    finally:
        p.close()


def test_register_overlap_refused(ec):
    """Two registrations must not share a page (the runtime maps pages
    whole; unregistering one would unmap the other's): a range overlapping
    a live one, or inside the pinned pool, is -EEXIST, synchronously for
    both calls; after the first is unregistered the second goes through."""
    import errno
    import mmap
    lib = ec.ec_method.lib
    m = mmap.mmap(-1, 16 << 10)
    a = np.frombuffer(m, np.uint8)
    base = a.ctypes.data
    assert lib.ec_method_host_register(base, 8 << 10) == 0
    try:
        assert lib.ec_method_host_register(base + (4 << 10), 8 << 10) == -errno.EEXIST
        assert lib.ec_method_host_register(base + (8 << 10) - 1, 100) == -errno.EEXIST
        assert lib.ec_method_host_register_async(base + 100, 4 << 10) == -errno.EEXIST
        pb = ec.PoolBuffer(1 << 20)
        if pb.pooled:
            assert lib.ec_method_host_register(pb.array.ctypes.data, 1 << 20) == -errno.EEXIST
        pb.free()
    finally:
        assert lib.ec_method_host_unregister(base) == 0
    assert lib.ec_method_host_register(base + (4 << 10), 8 << 10) == 0
    assert lib.ec_method_host_unregister(base + (4 << 10)) == 0
    del a


def test_register_errors(ec):
    import ctypes
    lib = ec.ec_method.lib
    a = np.empty(1 << 20, np.uint8)
    assert lib.ec_method_host_register(None, 4096) == -22
    assert lib.ec_method_host_register(ctypes.c_void_p(a.ctypes.data), 0) == -22
    assert lib.ec_method_host_unregister(ctypes.c_void_p(a.ctypes.data)) == -22
    # the refused call's HIP error is reported, not left pending for the
    # caller's next HIP call (it once failed the next test's torch copy)
    import torch
    t = torch.empty(4096, dtype=torch.uint8, device="cuda")
    t.copy_(torch.from_numpy(a[:4096]))
    torch.cuda.synchronize()
    with ec.host_registered(a):
        pass


@pytest.mark.parametrize("spec", ["0", "0,0,7", "junk"])
def test_host_devices_env(spec):
    """EC_MI355X_HOST_DEVICES restricts the host-buffer path to a device
    list (ec_device.hip host_devices_from_env); out-of-range or unparsable
    entries are ignored and an empty set falls back to every device.  The
    variable is read once per process, so each case runs in a child."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import sys, numpy as np
sys.path.insert(0, %r); sys.path.insert(0, %r)
import torch, glusterfs_amd as g, oracle as O
k, n, nst = 4, 6, 4096
data = O.fill_xorshift(512 * k * nst)
frags = [np.empty(512 * nst, np.uint8) for _ in range(n)]
with g.ECMatrixList(k, n) as L:
    L.encode_batch(nst, data, frags)
want = O.encode(k, n, data)
assert all(np.array_equal(a, b) for a, b in zip(frags, want))
print("ok")
''' % (root, os.path.join(root, "oracle"))
    env = dict(os.environ, EC_MI355X_HOST_DEVICES=spec, EC_SPLIT_MIN_MB="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=110)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-2000:]


def _attr_queries(kind):
    """HIP pointer-attribute queries made by 4 host encodes of 8 stripes on
    `kind` buffers (EC_MI355X_DEBUG=1 prints the count at exit)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import numpy as np, glusterfs_amd as g\n"
        "L = g.ECMatrixList(4, 6)\n"
        "if %r == 'pinned':\n"
        "    bufs = [g.PinnedArray(512 * 4 * 8)] + [g.PinnedArray(512 * 8) for _ in range(6)]\n"
        "    arrs = [b.array for b in bufs]\n"
        "else:\n"
        "    arrs = [np.zeros(512 * 4 * 8, np.uint8)] + [np.zeros(512 * 8, np.uint8) for _ in range(6)]\n"
        "for _ in range(4):\n"
        "    L.encode_batch(8, arrs[0], arrs[1:])\n" % kind)
    # (a lifetime longer than the run: the entries' expiry is
    # test_gpu_guards.py's subject)
    env = dict(os.environ, EC_MI355X_DEBUG="1", EC_MI355X_QUIET="1", EC_HOSTPAGE_MS="10000")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stderr.splitlines() if "pointer queries" in l][-1]
    return int(line.split("queries:")[1].split()[0])


def test_pinned_pages_are_queried_every_call(ec):
    """The per-thread host-page cache (ec_device.hip ecd_ptr_device) keeps
    only pages the HIP runtime does not know.  Pinned host pages come from
    the runtime's GPU virtual range: freed, their addresses are handed out
    again, also for device buffers -- a cached "host" verdict then routed a
    device-resident call as a host one (-EINVAL, r02z).  So pinned buffers
    are queried on every call, pageable ones once."""
    pinned = _attr_queries("pinned")
    pageable = _attr_queries("pageable")
    assert pinned >= 4 * 7, pinned          # every buffer, every call
    assert pageable <= 7 + 2, pageable      # first call only


_MAP_CHILD = r"""
import mmap, sys
sys.path[:0] = [%(root)r, %(oracle)r]
import numpy as np, glusterfs_amd as g, oracle as O
L = g.ECMatrixList(4, 6)
data = np.random.default_rng(3).integers(0, 256, 512 * 4 * 8, dtype=np.uint8)
frags = [np.zeros(512 * 8, np.uint8) for _ in range(6)]
want = O.encode(4, 6, data)
for i in range(%(calls)d):
    if i == %(reg_at)d:      # the library registers memory: cached verdicts go stale
        m = mmap.mmap(-1, 1 << 20)
        a = np.frombuffer(m, np.uint8)
        assert g.ec_method.lib.ec_method_host_register(a.ctypes.data, a.size) == 0
        assert g.ec_method.lib.ec_method_host_unregister(a.ctypes.data) == 0
        del a
    L.encode_batch(8, data, frags)
    assert all(np.array_equal(f, w) for f, w in zip(frags, want))
"""


def _map_queries(calls, reg_at=-1, ttl_ms="10000"):
    """hipHostGetDevicePointer ranges checked by `calls` GPU-routed host
    encodes on 7 pageable buffers (EC_MI355X_DEBUG=1 prints the count)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _MAP_CHILD % dict(root=root, oracle=os.path.join(root, "oracle"), calls=calls,
                             reg_at=reg_at)
    env = dict(os.environ, EC_MI355X_DEBUG="1", EC_MI355X_QUIET="1", EC_HOSTPAGE_MS=ttl_ms,
               EC_GPU_ALWAYS="1")
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stderr.splitlines() if "pointer queries" in l][-1]
    return int(line.split("attribute,")[1].split()[0])


def test_unmapped_ranges_cached_until_a_registration(ec):
    """ec_device.hip mapped(): a range found not mapped is not asked about
    again (the queries serialise in the HIP runtime under many client
    threads) until the lifetime ends or the library registers memory; a
    mapped verdict is never cached.  Every call is checked against the
    oracle."""
    never = _map_queries(20, ttl_ms="0")
    once = _map_queries(20)
    again = _map_queries(20, reg_at=10)
    assert never >= 20 * 7, never
    assert once <= 2 * 7 + 2, once                 # the first call's ranges only
    assert again >= once + 7, (once, again)         # asked again after the registration
