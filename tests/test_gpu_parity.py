"""GPU parity: the HIP kernels through the C ABI vs the CPU oracle.

Bit-exact comparison (integer GF(2^8) work: no tolerance).  Small seeded
inputs go through both the oracle and the library; inputs are host numpy
buffers (PCIe path) or torch device tensors (device-resident path).
"""
import itertools

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


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def rand_bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


GEOMS = [(2, 3), (3, 4), (4, 5), (4, 6), (6, 8), (8, 10), (8, 12), (10, 13), (16, 18),
         (16, 20), (16, 31)]


@pytest.mark.parametrize("k,n", GEOMS)
@pytest.mark.parametrize("nstripes", [1, 7, 64, 133])
def test_encode_host_matches_oracle(ec, oracle, k, n, nstripes):
    data = rand_bytes(CHUNK * k * nstripes, seed=k * 1000 + n * 10 + nstripes)
    want = oracle.encode(k, n, data)
    with ec.ECMatrixList(k, n) as L:
        got = [np.full(CHUNK * nstripes, 0xA5, dtype=np.uint8) for _ in range(n)]
        outs = list(got)
        L.encode(data.size, data, outs)
        for i in range(n):
            assert np.array_equal(got[i], want[i]), "fragment %d" % i


@pytest.mark.parametrize("k,n", [(2, 3), (4, 6), (8, 12), (16, 20), (5, 7)])
def test_encode_device_matches_oracle(ec, oracle, torch_cuda, k, n):
    torch = torch_cuda
    nstripes = 1000
    data = rand_bytes(CHUNK * k * nstripes, seed=11 + k)
    want = oracle.encode(k, n, data)
    din = torch.from_numpy(data).cuda()
    douts = [torch.empty(CHUNK * nstripes, dtype=torch.uint8, device="cuda") for _ in range(n)]
    with ec.ECMatrixList(k, n) as L:
        L.encode_batch(nstripes, din, douts)  # device pointers -> device path
        for i in range(n):
            assert np.array_equal(douts[i].cpu().numpy(), want[i]), "fragment %d" % i


def _decode_case(ec, oracle, L, k, n, rows, frags, nstripes, device=False):
    import torch
    want = oracle.decode(k, rows, [frags[r - 1] for r in rows])
    mask = sum(1 << (r - 1) for r in rows)
    if device:
        ins = [torch.from_numpy(frags[r - 1]).cuda() for r in rows]
        out = torch.empty(CHUNK * k * nstripes, dtype=torch.uint8, device="cuda")
        L.decode_batch(nstripes, mask, rows, ins, out)
        got = out.cpu().numpy()
    else:
        out = np.zeros(CHUNK * k * nstripes, dtype=np.uint8)
        L.decode(CHUNK * nstripes, mask, rows, [frags[r - 1] for r in rows], out)
        got = out
    assert np.array_equal(got, want), rows


@pytest.mark.parametrize("k,n", [(2, 3), (3, 4), (4, 6), (8, 12)])
def test_decode_all_masks_random_fragments(ec, oracle, k, n):
    """Fragments are random (not codewords): checks the full linear map."""
    nstripes = 9
    frags = [rand_bytes(CHUNK * nstripes, seed=100 + i) for i in range(n)]
    with ec.ECMatrixList(k, n) as L:
        for rows in itertools.combinations(range(1, n + 1), k):
            _decode_case(ec, oracle, L, k, n, list(rows), frags, nstripes)


@pytest.mark.parametrize("k,n", [(16, 20), (16, 18), (10, 13)])
def test_decode_sampled_masks(ec, oracle, k, n):
    nstripes = 17
    frags = [rand_bytes(CHUNK * nstripes, seed=300 + i) for i in range(n)]
    combos = list(itertools.combinations(range(1, n + 1), k))
    rng = np.random.default_rng(5)
    with ec.ECMatrixList(k, n) as L:
        for idx in rng.choice(len(combos), size=min(60, len(combos)), replace=False):
            _decode_case(ec, oracle, L, k, n, list(combos[idx]), frags, nstripes)


@pytest.mark.parametrize("k,n", [(4, 6), (8, 12), (16, 20)])
def test_decode_device_roundtrip(ec, oracle, torch_cuda, k, n):
    nstripes = 777
    data = rand_bytes(CHUNK * k * nstripes, seed=3)
    frags = oracle.encode(k, n, data)
    with ec.ECMatrixList(k, n) as L:
        rows = list(range(n - k + 1, n + 1))      # the first r bricks missing
        _decode_case(ec, oracle, L, k, n, rows, frags, nstripes, device=True)
        rows = sorted(np.random.default_rng(1).choice(n, k, replace=False) + 1)
        _decode_case(ec, oracle, L, k, n, [int(r) for r in rows], frags, nstripes, device=True)


def test_empty_and_cache(ec, oracle):
    k, n = 4, 6
    with ec.ECMatrixList(k, n, max=3) as L:
        L.encode(0, np.zeros(0, np.uint8), [np.zeros(0, np.uint8)] * n)
        L.decode(0, 0x0F, [1, 2, 3, 4], [np.zeros(0, np.uint8)] * k, np.zeros(0, np.uint8))
        frags = [rand_bytes(CHUNK * 3, seed=i) for i in range(n)]
        for rows in itertools.combinations(range(1, 7), 4):   # 15 masks > cache of 3
            _decode_case(ec, oracle, L, k, n, list(rows), frags, 3)
        assert L.count <= 3


def test_invalid_arguments(ec):
    with ec.ECMatrixList(4, 6) as L:
        buf = np.zeros(CHUNK * 4, np.uint8)
        with pytest.raises(OSError):   # mask with 3 bits
            L.decode(CHUNK, 0x07, [1, 2, 3], [buf] * 4, buf)
        with pytest.raises(OSError):   # rows inconsistent with mask
            L.decode(CHUNK, 0x0F, [1, 2, 3, 5], [buf] * 4, buf)
        with pytest.raises(OSError):   # size not a multiple of the chunk
            L.decode(100, 0x0F, [1, 2, 3, 4], [buf] * 4, buf)
    with pytest.raises(OSError):
        ec.ECMatrixList(8, 4)
    with pytest.raises(OSError):
        ec.ECMatrixList(17, 20)


def test_encode_advances_out_pointers(ec, oracle):
    """ec-method.c:405: each out[i] is advanced by size/k (ec_method_encode)."""
    import ctypes
    k, n, nst = 4, 6, 5
    data = rand_bytes(CHUNK * k * nst, seed=8)
    bufs = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n)]
    with ec.ECMatrixList(k, n) as L:
        ptrs = (ctypes.c_void_p * n)(*[b.ctypes.data for b in bufs])
        ec.ec_method.lib.ec_method_encode(ctypes.byref(L._list), data.size, data.ctypes.data,
                                          ptrs)
        for i in range(n):
            assert ptrs[i] == bufs[i].ctypes.data + CHUNK * nst
    want = oracle.encode(k, n, data)
    for i in range(n):
        assert np.array_equal(bufs[i], want[i])


@pytest.mark.parametrize("k,n,group", [(4, 6, 8), (4, 6, 16), (8, 12, 16), (8, 12, 64),
                                       (16, 20, 8), (3, 5, 32)])
def test_decode_mixed_patterns(ec, oracle, k, n, group):
    ngroups = 23
    nstripes = group * ngroups - 5          # ragged last group
    data = rand_bytes(CHUNK * k * nstripes, seed=21)
    frags = oracle.encode(k, n, data)
    rng = np.random.default_rng(4)
    pool = [sum(1 << int(b) for b in rng.choice(n, k, replace=False)) for _ in range(5)]
    masks = [pool[i] for i in rng.integers(0, len(pool), ngroups)]
    out = np.zeros(CHUNK * k * nstripes, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed(nstripes, group, masks, frags, out)
    assert np.array_equal(out, data)


@pytest.mark.parametrize("k,n", [(4, 6), (8, 12), (16, 20)])
def test_heal_regenerates_missing_fragments(ec, oracle, k, n):
    nstripes = 300
    data = rand_bytes(CHUNK * k * nstripes, seed=31)
    frags = oracle.encode(k, n, data)
    rows = list(range(n - k + 1, n + 1))               # good bricks: the last k
    mask = sum(1 << (r - 1) for r in rows)
    target = ((1 << n) - 1) & ~mask                     # regenerate the rest
    tgt = [i for i in range(n) if (target >> i) & 1]
    outs = [np.zeros(CHUNK * nstripes, np.uint8) for _ in tgt]
    with ec.ECMatrixList(k, n) as L:
        L.heal(nstripes, mask, [frags[r - 1] for r in rows], target, outs)
    for o, i in zip(outs, tgt):
        assert np.array_equal(o, frags[i]), "brick %d" % i


def test_concurrent_callers(ec, oracle):
    """Re-entrancy: many threads share one list (ec-method.c:206,250 lock)."""
    import threading
    k, n, nst = 4, 6, 40
    data = rand_bytes(CHUNK * k * nst, seed=77)
    frags = oracle.encode(k, n, data)
    errors = []
    with ec.ECMatrixList(k, n) as L:
        def worker(t):
            try:
                for rows in list(itertools.combinations(range(1, 7), 4))[t::4]:
                    out = np.zeros(data.size, np.uint8)
                    mask = sum(1 << (r - 1) for r in rows)
                    L.decode(CHUNK * nst, mask, list(rows), [frags[r - 1] for r in rows], out)
                    if not np.array_equal(out, data):
                        errors.append(rows)
                    enc = [np.zeros(CHUNK * nst, np.uint8) for _ in range(n)]
                    L.encode_batch(nst, data, enc)
                    if any(not np.array_equal(a, b) for a, b in zip(enc, frags)):
                        errors.append(("enc", t))
            except Exception as e:  # pragma: no cover
                errors.append(repr(e))
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
    assert not errors


def test_mixed_and_heal_device(ec, oracle, torch_cuda):
    torch = torch_cuda
    k, n, nst, group = 8, 12, 4096, 512
    data = rand_bytes(CHUNK * k * nst, seed=41)
    frags = oracle.encode(k, n, data)
    dfr = [torch.from_numpy(f).cuda() for f in frags]
    masks = [0xFF0, 0xEB5 | 0x0, 0x0FF, 0xF0F]
    masks = [m for m in masks if bin(m).count("1") == k]
    gp = torch.tensor([i % len(masks) for i in range(nst // group)], dtype=torch.uint8,
                      device="cuda")
    out = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed_device(0, None, nst, group, gp, masks, dfr, out)
        ec.sync_device(0)
        assert np.array_equal(out.cpu().numpy(), data)
        mask = 0xEB5
        good = [b for b in range(n) if (mask >> b) & 1]
        target = ((1 << n) - 1) & ~mask
        tgt = [b for b in range(n) if (target >> b) & 1]
        outs = [torch.empty(CHUNK * nst, dtype=torch.uint8, device="cuda") for _ in tgt]
        L.heal_device(0, None, nst, mask, [dfr[b] for b in good], target, outs)
        ec.sync_device(0)
        for o, b in zip(outs, tgt):
            assert np.array_equal(o.cpu().numpy(), frags[b])


def _distinct_masks(n, k, count, seed):
    rng = np.random.default_rng(seed)
    seen = []
    while len(seen) < count:
        m = sum(1 << int(b) for b in rng.choice(n, k, replace=False))
        if m not in seen:
            seen.append(m)
    return seen


@pytest.mark.parametrize("k,n,nmasks", [(16, 20, 40), (8, 12, 60), (16, 31, 50),
                                        (4, 6, 15)])
def test_decode_mixed_many_patterns_host(ec, oracle, k, n, nmasks):
    """More erasure masks than the 2 KiB kernel-argument segment holds
    (7 for 16+4, 28 for 8+4): the decode matrices go to a device table."""
    group, ngroups = 8, 2 * nmasks + 3
    nstripes = group * ngroups - 3
    data = rand_bytes(CHUNK * k * nstripes, seed=k * 7 + nmasks)
    frags = oracle.encode(k, n, data)
    pool = _distinct_masks(n, k, nmasks, seed=nmasks)
    masks = [pool[g % nmasks] for g in range(ngroups)]
    out = np.zeros(CHUNK * k * nstripes, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed(nstripes, group, masks, frags, out)
    assert np.array_equal(out, data)


def test_decode_mixed_too_many_patterns(ec, oracle):
    import errno
    k, n = 3, 12                     # C(12, 3) = 220 < 256: accepted
    pool = _distinct_masks(n, k, 220, seed=5)
    nst = 8 * len(pool)
    data = rand_bytes(CHUNK * k * nst, seed=6)
    frags = oracle.encode(k, n, data)
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed(nst, 8, pool, frags, out)
        assert np.array_equal(out, data)
    k, n = 4, 12                     # 257 distinct masks: -E2BIG
    pool = _distinct_masks(n, k, 257, seed=7)
    nst = 8 * len(pool)
    data = rand_bytes(CHUNK * k * nst, seed=8)
    frags = oracle.encode(k, n, data)
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        with pytest.raises(OSError) as ei:
            L.decode_mixed(nst, 8, pool, frags, out)
        assert ei.value.errno == errno.E2BIG


def test_mixed_device_table_cache(ec, oracle, torch_cuda):
    """Mixed decodes past the argument space reuse their device table across
    calls (ec_kernels.hip PatTableCache, 16 entries per device): 20 distinct
    sets of 12 masks of 16+4, cycled twice, so later calls hit entries and
    others evict them, and two threads on their own streams decode the same
    set concurrently.  Random fragments: every group is compared with the
    oracle's inverse."""
    import threading
    torch = torch_cuda
    k, n, group, per = 16, 20, 8, 12
    sets = [_distinct_masks(n, k, per, seed=300 + i) for i in range(20)]
    nst = group * per
    frags = [rand_bytes(CHUNK * nst, seed=900 + f) for f in range(n)]
    dfr = [torch.from_numpy(f).cuda() for f in frags]
    gp = torch.arange(per, dtype=torch.uint8, device="cuda")
    with ec.ECMatrixList(k, n) as L:
        for rep in range(2):
            for masks in sets:
                out = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
                L.decode_mixed_device(0, None, nst, group, gp, masks, dfr, out)
                ec.sync_device(0)
                _check_groups(oracle, k, group, nst, masks, frags, out.cpu().numpy())
        outs, errs = {}, []

        def worker(t):
            try:
                st = torch.cuda.Stream()
                o = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
                for _ in range(10):
                    L.decode_mixed_device(0, st.cuda_stream, nst, group, gp, sets[t % 3], dfr, o)
                st.synchronize()
                outs[t] = o.cpu().numpy()
            except Exception as e:                 # reported below
                errs.append(e)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        for t, o in outs.items():
            _check_groups(oracle, k, group, nst, sets[t % 3], frags, o)


def _check_groups(oracle, k, group, nst, masks, frags, out):
    for g, m in enumerate(masks):
        s0, s1 = g * group, min((g + 1) * group, nst)
        rows = oracle.mask_rows(m)
        want = oracle.decode(k, rows, [frags[r - 1][s0 * CHUNK:s1 * CHUNK] for r in rows])
        assert np.array_equal(out[s0 * CHUNK * k:s1 * CHUNK * k], want), \
            "group %d mask %#x" % (g, m)


@pytest.mark.parametrize("k,n,group,nmasks", [(4, 6, 1, 5), (4, 6, 2, 15), (8, 12, 4, 9),
                                              (16, 20, 1, 5), (16, 20, 2, 40), (3, 5, 4, 4),
                                              (10, 13, 1, 12)])
def test_decode_mixed_small_groups(ec, oracle, k, n, group, nmasks):
    """Pattern groups below one 8-stripe tile (1, 2, 4 stripes: the per-stripe
    waterfall kernel ec_combine_fine), incl. > 7 masks of 16+4 (device pattern
    table) and a ragged last group.  Random fragments, so every group is
    checked as the oracle's inverse applied to its bricks, not a round trip."""
    ngroups = 61
    nst = group * ngroups - (group - 1)
    frags = [rand_bytes(CHUNK * nst, seed=group * 97 + f) for f in range(n)]
    pool = _distinct_masks(n, k, nmasks, seed=group * 100 + k)
    rng = np.random.default_rng(group + k)
    masks = [pool[i] for i in rng.integers(0, nmasks, ngroups)]
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed(nst, group, masks, frags, out)
    _check_groups(oracle, k, group, nst, masks, frags, out)


@pytest.mark.parametrize("group", [0, 3, 12])
def test_decode_mixed_bad_group_size(ec, oracle, group):
    import errno
    k, n, nst = 4, 6, 48
    frags = [rand_bytes(CHUNK * nst, seed=f) for f in range(n)]
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        with pytest.raises(OSError) as ei:
            L.decode_mixed(nst, group, [0x3C] * nst, frags, out)
        assert ei.value.errno == errno.EINVAL


@pytest.mark.parametrize("k,n,group,nmasks", [(4, 6, 1, 15), (16, 20, 4, 30)])
def test_decode_mixed_small_groups_device(ec, oracle, torch_cuda, k, n, group, nmasks):
    torch = torch_cuda
    ngroups = 301
    nst = group * ngroups
    frags = [rand_bytes(CHUNK * nst, seed=group * 13 + f) for f in range(n)]
    dfr = [torch.from_numpy(f).cuda() for f in frags]
    pool = _distinct_masks(n, k, nmasks, seed=nmasks + 9)
    ids = np.random.default_rng(5).integers(0, nmasks, ngroups).astype(np.uint8)
    ids[-1] = 251                     # out of range: clamped to the last mask
    gp = torch.from_numpy(ids).cuda()
    out = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed_device(0, None, nst, group, gp, pool, dfr, out)
        ec.sync_device(0)
    masks = [pool[min(int(i), nmasks - 1)] for i in ids]
    _check_groups(oracle, k, group, nst, masks, frags, out.cpu().numpy())


@pytest.mark.parametrize("k,n,nmasks", [(16, 20, 100), (8, 12, 30)])
def test_decode_mixed_many_patterns_device(ec, oracle, torch_cuda, k, n, nmasks):
    torch = torch_cuda
    group = 16
    ngroups = 3 * nmasks
    nst = group * ngroups
    data = rand_bytes(CHUNK * k * nst, seed=nmasks + 1)
    frags = oracle.encode(k, n, data)
    dfr = [torch.from_numpy(f).cuda() for f in frags]
    masks = _distinct_masks(n, k, nmasks, seed=nmasks + 2)
    ids = np.random.default_rng(3).integers(0, nmasks, ngroups).astype(np.uint8)
    ids[-1] = 250                     # out of range: clamped to the last mask
    gp = torch.from_numpy(ids).cuda()
    out = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed_device(0, None, nst, group, gp, masks, dfr, out)
        ec.sync_device(0)
    assert np.array_equal(out.cpu().numpy(), data)


@pytest.mark.parametrize("k,n", [(16, 20), (16, 18), (10, 13), (8, 12)])
def test_decode_every_mask_random_fragments(ec, oracle, k, n):
    """Exhaustive erasure coverage: every k-of-n brick set (4845 for 16+4)
    decodes random (non-codeword) fragments exactly as the oracle's inverse,
    i.e. the full linear map, 256 masks per mixed call (8-stripe groups)."""
    group = 8
    allm = [sum(1 << b for b in c) for c in itertools.combinations(range(n), k)]
    with ec.ECMatrixList(k, n) as L:
        for c0 in range(0, len(allm), 256):
            masks = allm[c0:c0 + 256]
            nst = group * len(masks)
            frags = [rand_bytes(CHUNK * nst, seed=c0 * 31 + f) for f in range(n)]
            out = np.zeros(CHUNK * k * nst, np.uint8)
            L.decode_mixed(nst, group, masks, frags, out)
            span = CHUNK * group
            for g, m in enumerate(masks):
                rows = oracle.mask_rows(m)
                want = oracle.decode(k, rows, [frags[r - 1][g * span:(g + 1) * span]
                                               for r in rows])
                got = out[g * span * k:(g + 1) * span * k]
                assert np.array_equal(got, want), "mask %#x" % m


# --- device-resident kernels, exhaustively (the instantiations bench.py times) ---

def _device_decode_masks(ec, oracle, torch, k, n, masks, nst, seed, nthreads=1):
    """decode_batch on torch device buffers (ec_method_decode_device ->
    ec_combine<K,TS,NW,false,NTS>) for every mask, on random fragments, each
    output compared with the oracle's inverse applied to the same bricks."""
    frags = [rand_bytes(CHUNK * nst, seed + i) for i in range(n)]
    dfr = [torch.from_numpy(f).cuda() for f in frags]
    out = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
    with ec.ECMatrixList(k, n) as L:
        for m in masks:
            rows = oracle.mask_rows(m)
            out.fill_(0xA5)
            L.decode_batch(nst, m, rows, [dfr[r - 1] for r in rows], out)
            want = oracle.decode(k, rows, [frags[r - 1] for r in rows], nthreads=nthreads)
            assert np.array_equal(out.cpu().numpy(), want), "mask %#x" % m


@pytest.mark.parametrize("k,n,nst", [(4, 6, 77), (8, 12, 61), (2, 3, 40), (3, 5, 19)])
def test_decode_device_every_mask(ec, oracle, torch_cuda, k, n, nst):
    """All 15 masks of 4+2 and all 495 of 8+4 on the device-resident path."""
    masks = [sum(1 << b for b in c) for c in itertools.combinations(range(n), k)]
    _device_decode_masks(ec, oracle, torch_cuda, k, n, masks, nst, seed=k * 31 + n)


def test_decode_device_every_mask_16p4(ec, oracle, torch_cuda):
    """Every one of the 4845 masks of 16+4 on the device-resident path (the
    k = 16 kernel bench.py times), 13 stripes: one full 8-stripe tile and a
    ragged one."""
    k, n = 16, 20
    allm = [sum(1 << b for b in c) for c in itertools.combinations(range(n), k)]
    assert len(allm) == 4845
    _device_decode_masks(ec, oracle, torch_cuda, k, n, allm, 13, seed=1604)


@pytest.mark.parametrize("mask", [0xFF0, 0xEB5])
def test_decode_device_8p4_large_batch(ec, oracle, torch_cuda, mask):
    """More than 131,072 stripes of 8+4 (a full decode past the 128K-stripe
    switch of round 1; since r02z every 8+4 full decode runs the 16-wave
    instantiation, ec_kernels.hip launch_combine_k)."""
    _device_decode_masks(ec, oracle, torch_cuda, 8, 12, [mask], (1 << 17) + 77, seed=812,
                         nthreads=8)


def test_encode_device_large_batches(ec, oracle, torch_cuda):
    """Device encode at sizes past one grid wave, every specialised geometry;
    8+4 on both sides of the 128K-stripe switch to the tile encoder
    (ec_kernels.hip ecdk_encode_vander)."""
    torch = torch_cuda
    for k, n, nst in ((4, 6, 300007), (8, 12, 70001), (8, 12, (1 << 17) + 3), (16, 20, 20011),
                      (16, 20, 3)):
        data = rand_bytes(CHUNK * k * nst, seed=nst)
        want = oracle.encode(k, n, data, nthreads=8)
        din = torch.from_numpy(data).cuda()
        outs = [torch.empty(CHUNK * nst, dtype=torch.uint8, device="cuda") for _ in range(n)]
        with ec.ECMatrixList(k, n) as L:
            L.encode_batch(nst, din, outs)
        for i in range(n):
            assert np.array_equal(outs[i].cpu().numpy(), want[i]), (k, n, i)


# --- argument guards --------------------------------------------

def test_decode_mixed_null_fragment_rejected(ec, torch_cuda):
    """A mask that reads a brick whose fragment is NULL fails with EINVAL on
    the host and device paths instead of faulting the device."""
    import errno
    torch = torch_cuda
    k, n, nst = 4, 6, 64
    frags = [rand_bytes(CHUNK * nst, f) for f in range(n)]
    frags[0] = None                                  # brick 0 absent
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed(nst, 8, [0x3C] * 8, frags, out)          # 0x3C reads bricks 2-5
        with pytest.raises(OSError) as ei:
            L.decode_mixed(nst, 8, [0x3C, 0x0F] * 4, frags, out)  # 0x0F reads brick 0
        assert ei.value.errno == errno.EINVAL
        dfr = [None if f is None else torch.from_numpy(f).cuda() for f in frags]
        dout = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
        gp = torch.zeros(nst // 8, dtype=torch.uint8, device="cuda")
        with pytest.raises(OSError) as ei:
            L.decode_mixed_device(0, None, nst, 8, gp, [0x0F], dfr, dout)
        assert ei.value.errno == errno.EINVAL


def test_mixed_host_device_buffers_rejected(ec, torch_cuda):
    import errno
    torch = torch_cuda
    k, n, nst = 4, 6, 16
    with ec.ECMatrixList(k, n) as L:
        din = [torch.zeros(CHUNK * nst, dtype=torch.uint8, device="cuda") for _ in range(k)]
        hout = [np.zeros(CHUNK * nst, np.uint8) for _ in range(2)]
        with pytest.raises(OSError) as ei:              # device in, host out
            L.heal(nst, 0x3C, din, 0x03, hout)
        assert ei.value.errno == errno.EINVAL
        hin = [np.zeros(CHUNK * nst, np.uint8) for _ in range(k)]
        hin[3] = din[3]
        with pytest.raises(OSError) as ei:              # one device input among host ones
            L.heal(nst, 0x3C, hin, 0x03, hout)
        assert ei.value.errno == errno.EINVAL
        user = torch.zeros(CHUNK * k * 3, dtype=torch.uint8, device="cuda")
        with pytest.raises(OSError) as ei:              # device user data, host fragments
            L.writev_encode(0, user, None, None, [np.zeros(CHUNK * 3, np.uint8)] * n)
        assert ei.value.errno == errno.EINVAL


def test_decode_mixed_group_larger_than_call(ec, oracle):
    """group_stripes far above nstripes: one group, staging sized by the data."""
    k, n, nst = 4, 6, 100
    data = rand_bytes(CHUNK * k * nst, 12)
    frags = oracle.encode(k, n, data)
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed(nst, 1 << 20, [0xF0 >> 2], frags, out)
    assert np.array_equal(out, data)


@pytest.mark.parametrize("k,n,group", [(4, 6, 1), (4, 6, 2), (8, 12, 1), (8, 12, 2), (3, 5, 1)])
def test_decode_mixed_short_runs(ec, oracle, k, n, group):
    """Sorted-slot runs of 1-3 stripes: each pattern's run is padded to 8
    slots and the narrow kernels take 4-slot tiles, so whole tiles are
    padding (round 3: they looked their pattern up at slot ~0 and faulted).
    Every mask appears 1-3 times; checked group by group against the
    oracle's inverse."""
    import math
    import torch
    nmasks = min(15, math.comb(n, k))
    pool = _distinct_masks(n, k, nmasks, seed=group * 7 + k)
    ids = []
    rng = np.random.default_rng(k + group)
    for m in range(nmasks):
        ids += [m] * int(rng.integers(1, 4))
    rng.shuffle(ids)
    ngroups = len(ids)
    nst = group * ngroups
    frags = [rand_bytes(CHUNK * nst, seed=500 + f) for f in range(n)]
    masks = [pool[i] for i in ids]
    out = np.zeros(CHUNK * k * nst, np.uint8)
    with ec.ECMatrixList(k, n) as L:
        L.decode_mixed(nst, group, masks, frags, out)
        _check_groups(oracle, k, group, nst, masks, frags, out)
        dfr = [torch.from_numpy(f).cuda() for f in frags]
        gp = torch.tensor(ids, dtype=torch.uint8, device="cuda")
        dout = torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda")
        L.decode_mixed_device(0, None, nst, group, gp, pool, dfr, dout)
        ec.sync_device(0)
        _check_groups(oracle, k, group, nst, masks, frags, dout.cpu().numpy())
