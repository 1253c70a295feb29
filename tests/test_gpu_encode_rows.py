"""ec_method_encode_rows on the GPU: the fragments of the bricks in row_mask
only (a heal write goes to heal->bad only, ec-heal.c:327-329, yet
ec_writev_encode computes all n, ec-inode-write.c:2125-2138).  Host buffers
(EC_GPU_ALWAYS=1, tests/conftest.py) run the device layer's generic encode:
the persistent zero-copy combine with the selected encode-matrix rows as its
pattern (k = 16 too while 2k + m tiles fit the CU's 160 KiB of LDS, i.e. up
to 7 rows), read in place when pinned and
through the staging slots when pageable; device buffers run ec_combine.  Every
case is compared bit for bit with the oracle's full encode (the checker)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 512
GEOS = [(2, 3), (4, 6), (8, 12), (16, 20)]


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


def masks_for(n):
    ms = {1, 1 << (n - 1), 0b11, (1 << (n - 1)) - 1}
    ms |= {int(m) for m in np.random.default_rng(n).integers(1, (1 << n) - 1, 3)}
    ms.discard((1 << n) - 1)
    return sorted(ms)


@pytest.mark.parametrize("k,n", GEOS)
def test_encode_rows_host_pageable(oracle, k, n):
    import glusterfs_amd as g
    s0 = g.ec_method.stats()
    with g.ECMatrixList(k, n) as L:
        for nst in (5, 1031, 4100):
            data = rnd(CHUNK * k * nst, nst + k)
            want = oracle.encode(k, n, data)
            for m in masks_for(n):
                outs = [np.full(CHUNK * nst, 0x5A, np.uint8) for _ in range(n)]
                L.encode_rows(data.size, data, m, [o if (m >> i) & 1 else None
                                                   for i, o in enumerate(outs)])
                for i in range(n):
                    if (m >> i) & 1:
                        assert np.array_equal(outs[i], want[i]), (k, n, nst, hex(m), i)
                    else:
                        assert (outs[i] == 0x5A).all()
    s1 = g.ec_method.stats()
    assert s1["gpu_calls"] > s0["gpu_calls"]
    assert s1["cpu_fallbacks"] == s0["cpu_fallbacks"]   # no device error redone on the CPU


@pytest.mark.parametrize("k,n", GEOS)
def test_encode_rows_host_pinned(oracle, k, n):
    """Pinned input and outputs: the zero-copy path, several tiles per block
    of the persistent kernel (4100 stripes)."""
    import glusterfs_amd as g
    lib = g.ec_method.lib
    nst = 4100
    S, fl = CHUNK * k * nst, CHUNK * nst
    ptrs = []

    def pinned(nb):
        p = lib.ec_method_host_alloc(nb)
        assert p
        ptrs.append(p)
        return p, np.ctypeslib.as_array((ctypes.c_uint8 * nb).from_address(p))

    s0 = g.ec_method.stats()
    try:
        ip, ia = pinned(S)
        ia[:] = rnd(S, 77)
        want = oracle.encode(k, n, ia.copy())
        outs = [pinned(fl) for _ in range(n)]
        with g.ECMatrixList(k, n) as L:
            for m in masks_for(n):
                for _, a in outs:
                    a[:] = 0x5A
                L.encode_rows(S, ip, m, [p if (m >> i) & 1 else None
                                         for i, (p, _) in enumerate(outs)])
                for i, (_, a) in enumerate(outs):
                    if (m >> i) & 1:
                        assert np.array_equal(a, want[i]), (k, n, hex(m), i)
                    else:
                        assert (a == 0x5A).all()
    finally:
        for p in ptrs:
            lib.ec_method_host_free(p)
    assert g.ec_method.stats()["cpu_fallbacks"] == s0["cpu_fallbacks"]


@pytest.mark.parametrize("k,n", GEOS)
def test_encode_rows_device(oracle, k, n):
    import torch
    import glusterfs_amd as g
    nst = 1031
    data = rnd(CHUNK * k * nst, 3 * k)
    want = oracle.encode(k, n, data)
    din = torch.from_numpy(data).cuda()
    with g.ECMatrixList(k, n) as L:
        for m in masks_for(n):
            outs = [torch.full((CHUNK * nst,), 0x5A, dtype=torch.uint8, device="cuda")
                    for _ in range(n)]
            L.encode_rows(data.size, din, m, [o if (m >> i) & 1 else None
                                              for i, o in enumerate(outs)])
            for i in range(n):
                got = outs[i].cpu().numpy()
                if (m >> i) & 1:
                    assert np.array_equal(got, want[i]), (k, n, hex(m), i)
                else:
                    assert (got == 0x5A).all()


@pytest.mark.parametrize("k,n", GEOS)
def test_encode_rows_device_async(oracle, k, n):
    """ec_method_encode_rows_device on a side stream, then synchronised."""
    import torch
    import glusterfs_amd as g
    nst = 777
    data = rnd(CHUNK * k * nst, 5 * k)
    want = oracle.encode(k, n, data)
    din = torch.from_numpy(data).cuda()
    st = torch.cuda.Stream()
    with g.ECMatrixList(k, n) as L:
        m = masks_for(n)[-1]
        outs = [torch.full((CHUNK * nst,), 0x5A, dtype=torch.uint8, device="cuda")
                for _ in range(n)]
        torch.cuda.synchronize()
        L.encode_rows_device(0, st.cuda_stream, nst, din, m,
                             [o if (m >> i) & 1 else None for i, o in enumerate(outs)])
        st.synchronize()
        for i in range(n):
            got = outs[i].cpu().numpy()
            if (m >> i) & 1:
                assert np.array_equal(got, want[i]), (k, n, hex(m), i)
            else:
                assert (got == 0x5A).all()
        with pytest.raises(OSError):
            L.encode_rows_device(0, st.cuda_stream, nst, din, 1 << n, outs)


@pytest.mark.parametrize("k,r,rows", [(16, 8, 20), (4, 3, 6), (8, 5, 12), (2, 2, 3)])
@pytest.mark.parametrize("kind", ["pinned", "pageable"])
def test_encode_rows_count_of_a_specialised_geometry(oracle, k, r, rows, kind):
    """Regression (tools/fuzz_api.py, r04u): a row-masked encode whose row
    count equals the n of a geometry with a specialised encoder (20 rows of
    a 16+8 volume, 6 of a 4+3, ...) took that encoder, i.e. the first n
    Vandermonde rows instead of the selected ones.  The host path now always
    runs the generic combination with the selected rows."""
    import glusterfs_amd as g
    n = k + r
    nst = 1031
    data = rnd(CHUNK * k * nst, k * 13 + r)
    want = oracle.encode(k, n, data)
    rng = np.random.default_rng(rows)
    keep = []
    try:
        def buf(nb):
            if kind == "pinned":
                p = g.PinnedArray(nb)
                keep.append(p)
                return p.array
            return np.empty(nb, np.uint8)
        src = buf(data.size)
        src[:] = data
        with g.ECMatrixList(k, n) as L:
            for _ in range(3):
                pick = sorted(rng.choice(n, rows, replace=False))
                if list(pick) == list(range(rows)):
                    pick = list(range(n - rows, n))
                m = sum(1 << int(b) for b in pick)
                outs = [buf(CHUNK * nst) if (m >> i) & 1 else None for i in range(n)]
                L.encode_rows(data.size, src, m, outs)
                for i, o in enumerate(outs):
                    if o is not None:
                        assert np.array_equal(o, want[i]), (k, n, hex(m), i)
    finally:
        for p in keep:
            p.free()
