"""The library's CPU engine (glusterfs_amd/csrc/ec_cpu*.c) against the oracle.

The engine is product code: it codes host buffers on nodes without a gfx950
GPU, for cpu-extensions = none / x64 / sse / avx, below the CPU/GPU
crossover and as the fallback after a device error.  It is checked here bit
for bit against the oracle (test infrastructure) for every ISA level the
host supports (gen = none -> base x86-64, avx2, avx512), on random (non-
codeword) fragments, so the full linear maps are compared, not round trips.
No GPU is needed: these run in the CPU suite.
"""
import itertools

import numpy as np
import pytest

CHUNK = 512
GENS = ["none", "avx2", "avx512"]


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


@pytest.fixture(scope="module")
def ec():
    import glusterfs_amd as g
    return g


def _isa_ok(ec, gen):
    with ec.ECMatrixList(2, 3, gen=gen) as L:
        eng = L.engine
    assert eng.startswith("cpu/")
    if gen == "avx512" and eng != "cpu/avx512":
        pytest.skip("host has no AVX-512")
    if gen == "avx2" and eng not in ("cpu/avx2",):
        pytest.skip("host has no AVX2")
    return eng


@pytest.mark.parametrize("gen", GENS)
@pytest.mark.parametrize("k,n", [(2, 3), (3, 4), (4, 6), (6, 8), (8, 12), (10, 13), (16, 20),
                                 (16, 31)])
def test_encode_matches_oracle(ec, oracle, gen, k, n):
    _isa_ok(ec, gen)
    for nst in (1, 5, 33):
        data = rnd(CHUNK * k * nst, k * 100 + nst)
        want = oracle.encode(k, n, data)
        with ec.ECMatrixList(k, n, gen=gen) as L:
            outs = [np.full(CHUNK * nst, 0x5A, np.uint8) for _ in range(n)]
            L.encode(data.size, data, list(outs))
        for i in range(n):
            assert np.array_equal(outs[i], want[i]), (gen, k, n, nst, i)


@pytest.mark.parametrize("gen", GENS)
@pytest.mark.parametrize("k,n", [(2, 3), (4, 6), (8, 12)])
def test_decode_every_mask(ec, oracle, gen, k, n):
    _isa_ok(ec, gen)
    nst = 6
    frags = [rnd(CHUNK * nst, 40 + f) for f in range(n)]
    with ec.ECMatrixList(k, n, gen=gen) as L:
        for rows in itertools.combinations(range(1, n + 1), k):
            rows = list(rows)
            out = np.zeros(CHUNK * k * nst, np.uint8)
            L.decode(CHUNK * nst, sum(1 << (r - 1) for r in rows), rows,
                     [frags[r - 1] for r in rows], out)
            assert np.array_equal(out, oracle.decode(k, rows, [frags[r - 1] for r in rows])), \
                rows


@pytest.mark.parametrize("gen", GENS)
@pytest.mark.parametrize("k,n", [(16, 20), (16, 31), (10, 13)])
def test_decode_sampled_masks(ec, oracle, gen, k, n):
    _isa_ok(ec, gen)
    nst = 3
    frags = [rnd(CHUNK * nst, 70 + f) for f in range(n)]
    rng = np.random.default_rng(k + n)
    with ec.ECMatrixList(k, n, gen=gen) as L:
        for _ in range(40):
            rows = sorted(int(r) + 1 for r in rng.choice(n, k, replace=False))
            out = np.zeros(CHUNK * k * nst, np.uint8)
            L.decode(CHUNK * nst, sum(1 << (r - 1) for r in rows), rows,
                     [frags[r - 1] for r in rows], out)
            assert np.array_equal(out, oracle.decode(k, rows, [frags[r - 1] for r in rows]))


@pytest.mark.parametrize("k,n,group,nmasks", [(4, 6, 1, 15), (8, 12, 8, 40), (16, 20, 2, 20),
                                              (16, 20, 64, 9)])
def test_decode_mixed(ec, oracle, k, n, group, nmasks):
    ng = 37
    nst = group * ng - (group > 1)
    frags = [rnd(CHUNK * nst, 90 + f) for f in range(n)]
    rng = np.random.default_rng(group)
    pool = []
    while len(pool) < nmasks:
        m = sum(1 << int(b) for b in rng.choice(n, k, replace=False))
        if m not in pool:
            pool.append(m)
    masks = [pool[i] for i in rng.integers(0, nmasks, ng)]
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n, gen="none") as L:
        L.decode_mixed(nst, group, masks, frags, out)
    for g_, m in enumerate(masks):
        s0, s1 = g_ * group, min((g_ + 1) * group, nst)
        rows = oracle.mask_rows(m)
        want = oracle.decode(k, rows, [frags[r - 1][s0 * CHUNK:s1 * CHUNK] for r in rows])
        assert np.array_equal(out[s0 * CHUNK * k:s1 * CHUNK * k], want), (g_, hex(m))


def _masks(n, k, count, seed):
    rng = np.random.default_rng(seed)
    pool = []
    while len(pool) < count:
        m = sum(1 << int(b) for b in rng.choice(n, k, replace=False))
        if m not in pool:
            pool.append(m)
    return pool


def test_decode_mixed_repeated_sets_across_volumes(ec, oracle):
    """The per-thread memo of mixed-call pattern sets (ec_method.c
    pattern_set, r05): the same sets again and again (memo hits), sets
    larger than the volume's decode-matrix cache, volumes of different k
    interleaved on one thread (the memo's buffers are shared and grow), and
    a volume torn down and re-created in the same ec_matrix_list_t (a new
    serial: no stale hit).  Every group against the oracle."""
    geos = [(4, 6), (16, 20), (8, 12)]
    group, ng = 2, 24
    nst = group * ng
    frags = {kn: [rnd(CHUNK * nst, 300 + 31 * kn[0] + f) for f in range(kn[1])] for kn in geos}
    counts = {(4, 6): (3, 9, 15), (16, 20): (3, 12, 45), (8, 12): (3, 12, 45)}  # C(6, 4) = 15
    sets = {kn: [_masks(kn[1], kn[0], c, seed=c + kn[0]) for c in counts[kn]] for kn in geos}
    rng = np.random.default_rng(9)

    def check(L, kn, masks):
        k, n = kn
        gm = [masks[int(i)] for i in rng.integers(0, len(masks), ng)]
        out = np.zeros(CHUNK * k * nst, np.uint8)
        L.decode_mixed(nst, group, gm, frags[kn], out)
        for g_, m in enumerate(gm):
            s0, s1 = g_ * group, (g_ + 1) * group
            rows = oracle.mask_rows(m)
            want = oracle.decode(k, rows, [frags[kn][r - 1][s0 * CHUNK:s1 * CHUNK] for r in rows])
            assert np.array_equal(out[s0 * CHUNK * k:s1 * CHUNK * k], want), (kn, g_, hex(m))

    vols = {kn: ec.ECMatrixList(kn[0], kn[1], gen="none") for kn in geos}
    try:
        for it in range(30):
            kn = geos[it % 3]
            check(vols[kn], kn, sets[kn][(it // 3) % 3])
            if it == 14:                                     # same struct, new volume
                vols[kn].fini()
                vols[kn] = ec.ECMatrixList(kn[0], kn[1], gen="none")
    finally:
        for L in vols.values():
            L.fini()


@pytest.mark.parametrize("k,n", [(4, 6), (8, 12), (16, 20)])
def test_heal(ec, oracle, k, n):
    nst = 20
    data = rnd(CHUNK * k * nst, 5)
    frags = oracle.encode(k, n, data)
    good = list(range(n - k, n))
    mask = sum(1 << b for b in good)
    target = ((1 << n) - 1) & ~mask
    outs = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n - k)]
    with ec.ECMatrixList(k, n, gen="avx") as L:
        L.heal(nst, mask, [frags[b] for b in good], target, outs)
    for i, o in enumerate(outs):
        assert np.array_equal(o, frags[i])


@pytest.mark.parametrize("k,n,head,size,old", [(4, 6, 0, 512 * 4 * 3, "none"),
                                               (4, 6, 1234, 5000, "both"),
                                               (8, 12, 7, 100, "head"),
                                               (8, 12, 4000, 9000, "tail"),
                                               (16, 20, 3, 8192 * 5 + 17, "both")])
def test_writev_merge(ec, oracle, k, n, head, size, old):
    S = CHUNK * k
    user = rnd(size, 3)
    oh = rnd(S, 4) if old in ("head", "both") else None
    ot = rnd(S, 5) if old in ("tail", "both") else None
    v = oracle.writev_merge(k, head, user, oh, ot)
    want = oracle.encode(k, n, v)
    nst = v.size // S
    with ec.ECMatrixList(k, n, gen="none") as L:
        outs = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n)]
        # the user data as an iovec list of 3 uneven pieces
        cuts = [0, size // 3, size // 3 + 1, size]
        L.writev_encode(head, [user[cuts[i]:cuts[i + 1]] for i in range(3)], oh, ot, outs)
    for i in range(n):
        assert np.array_equal(outs[i], want[i]), i


def test_engine_counters_and_guards(ec):
    import errno
    before = ec.stats()["cpu_calls"]
    k, n, nst = 4, 6, 8
    frags = [rnd(CHUNK * nst, f) for f in range(n)]
    frags[0] = None
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n, gen="none") as L:
        L.decode_mixed(nst, 8, [0x3C], frags, out)
        with pytest.raises(OSError) as ei:
            L.decode_mixed(nst, 8, [0x0F], frags, out)
        assert ei.value.errno == errno.EINVAL
    assert ec.stats()["cpu_calls"] == before + 1


@pytest.mark.parametrize("gen", GENS)
def test_every_constant_first_and_later_terms(ec, oracle, gen):
    """Every one of the 255 multiply programs, as the first term of a row
    (mul_c) and as a later one (mac_c): 16+31 masks are drawn until the
    inverses have covered all constants in both positions."""
    _isa_ok(ec, gen)
    k, n, nst = 16, 31, 1
    frags = [rnd(CHUNK * nst, 300 + f) for f in range(n)]
    rng = np.random.default_rng(255)
    first, later = set(), set()
    with ec.ECMatrixList(k, n, gen=gen) as L:
        for _ in range(2000):
            rows = sorted(int(r) + 1 for r in rng.choice(n, k, replace=False))
            inv = oracle.inverse_matrix(rows)
            new = False
            for row in inv:
                nz = [int(c) for c in row if c]
                new |= nz[0] not in first or any(c not in later for c in nz[1:])
                first.add(nz[0])
                later.update(nz[1:])
            if not new:
                continue
            out = np.zeros(CHUNK * k * nst, np.uint8)
            L.decode(CHUNK * nst, sum(1 << (r - 1) for r in rows), rows,
                     [frags[r - 1] for r in rows], out)
            assert np.array_equal(out, oracle.decode(k, rows, [frags[r - 1] for r in rows]))
            if len(first) == 255 and len(later) == 255:
                break
    assert len(first) == 255 and len(later) == 255, (len(first), len(later))


@pytest.mark.parametrize("gen", ["avx512"])
def test_large_calls_stream_outputs(ec, oracle, gen):
    """Calls whose outputs reach 16 MiB store them with streaming stores
    (AVX-512, 64-byte-aligned output bases; ec_cpu_kern.c stv): encode and
    full decode at that size, and a misaligned output base (regular stores),
    all bit-exact against the oracle."""
    _isa_ok(ec, gen)
    k, n = 4, 6
    nst = (16 << 20) // (CHUNK * k) + 3                  # > 16 MiB of decode output
    data = rnd(CHUNK * k * nst, seed=91)
    want = oracle.encode(k, n, data, nthreads=8)
    def aligned(nbytes):
        # 64-byte aligned, so the streaming-store path is really taken
        # (np.zeros bases are 16 bytes past a page)
        raw = np.zeros(nbytes + 64, np.uint8)
        off = (-raw.ctypes.data) % 64
        buf = raw[off:off + nbytes]
        assert buf.ctypes.data % 64 == 0
        return buf

    with ec.ECMatrixList(k, n, gen=gen) as L:
        frags = [aligned(CHUNK * nst) for _ in range(n)]
        L.encode_batch(nst, data, frags)
        for i in range(n):
            assert np.array_equal(frags[i], want[i]), i
        rows = [3, 4, 5, 6]
        out = aligned(data.size)
        L.decode_batch(nst, 0x3C, rows, [want[r - 1] for r in rows], out)
        assert np.array_equal(out, data)
        raw = aligned(data.size + 64)
        odd = raw[8:8 + data.size]               # misaligned: regular stores
        L.decode_batch(nst, 0x3C, rows, [want[r - 1] for r in rows], odd)
        assert np.array_equal(odd, data)


@pytest.mark.parametrize("gen", GENS)
@pytest.mark.parametrize("k,n", [(2, 3), (4, 6), (8, 12), (16, 20), (10, 13)])
def test_encode_rows_matches_oracle(ec, oracle, gen, k, n):
    """ec_method_encode_rows: only the bricks of row_mask are computed (the
    heal write of ec-heal.c:327-329 goes to heal->bad only), equal to those
    fragments of the oracle's full encode; the other buffers are untouched."""
    _isa_ok(ec, gen)
    rng = np.random.default_rng(k * 7 + n)
    masks = {1, 1 << (n - 1), (1 << (n - 1)) - 1}
    masks |= {int(m) for m in rng.integers(1, 1 << n, 6)}
    masks.discard((1 << n) - 1)
    nst = 9
    data = rnd(CHUNK * k * nst, k * 31 + n)
    want = oracle.encode(k, n, data)
    with ec.ECMatrixList(k, n, gen=gen) as L:
        for m in sorted(masks):
            outs = [np.full(CHUNK * nst, 0x5A, np.uint8) for _ in range(n)]
            arg = [outs[i] if (m >> i) & 1 else None for i in range(n)]
            L.encode_rows(data.size, data, m, arg)
            for i in range(n):
                if (m >> i) & 1:
                    assert np.array_equal(outs[i], want[i]), (gen, k, n, hex(m), i)
                else:
                    assert (outs[i] == 0x5A).all(), (gen, k, n, hex(m), i)


def test_encode_rows_pointer_contract(ec, oracle):
    """As ec_method_encode (ec-method.c:405), each selected out[i] advances by
    size/k; unselected entries (NULL here) stay as they are; an empty mask is
    a no-op and a full mask is ec_method_encode."""
    import ctypes
    k, n, nst = 4, 6, 3
    data = rnd(CHUNK * k * nst, 5)
    want = oracle.encode(k, n, data)
    with ec.ECMatrixList(k, n) as L:
        outs = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n)]
        m = 0b100110
        arr = (ctypes.c_void_p * n)(*[o.ctypes.data if (m >> i) & 1 else None
                                      for i, o in enumerate(outs)])
        ec.ec_method.lib.ec_method_encode_rows(ctypes.byref(L._list), data.size,
                                               data.ctypes.data, m, arr)
        for i in range(n):
            if (m >> i) & 1:
                assert arr[i] == outs[i].ctypes.data + data.size // k
                assert np.array_equal(outs[i], want[i])
            else:
                assert arr[i] is None
        ec.ec_method.lib.ec_method_encode_rows(ctypes.byref(L._list), data.size,
                                               data.ctypes.data, 0, arr)   # no-op
        full = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n)]
        L.encode_rows(data.size, data, (1 << n) - 1, full)
        for i in range(n):
            assert np.array_equal(full[i], want[i])
