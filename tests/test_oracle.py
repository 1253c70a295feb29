"""Pin the CPU oracle (oracle/ec_oracle.c) to the reference before trusting it.

* gf8_muladd_ref.npz: every gf8_muladd_XX routine of ec-code-c.c:20-11571,
  evaluated from the reference source text (tests/golden/gen_gf8_muladd.py).
* survey_appendix_c.json: inverse matrices and the zero-coefficient census
  recorded from the compiled reference in the survey session.
* independent restatements: a pure-Python GF(2^8) and Gauss-Jordan inverse.
"""
import itertools
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def py_gf_mul(a, b):
    r = 0
    for _ in range(8):
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
    return r


def py_gf_inv(a):
    for b in range(1, 256):
        if py_gf_mul(a, b) == 1:
            return b
    raise ZeroDivisionError


def py_inverse(mat):
    """Gauss-Jordan over GF(2^8) (independent of ec-method.c:38-72)."""
    k = len(mat)
    a = [list(r) + [int(i == j) for j in range(k)] for i, r in enumerate(mat)]
    for c in range(k):
        piv = next(r for r in range(c, k) if a[r][c])
        a[c], a[piv] = a[piv], a[c]
        inv = py_gf_inv(a[c][c])
        a[c] = [py_gf_mul(v, inv) for v in a[c]]
        for r in range(k):
            if r != c and a[r][c]:
                f = a[r][c]
                a[r] = [v ^ py_gf_mul(f, w) for v, w in zip(a[r], a[c])]
    return [r[k:] for r in a]


def test_gf8_muladd_matches_reference_programs(oracle):
    g = np.load(os.path.join(GOLD, "gf8_muladd_ref.npz"))
    out0, inp, exp = g["out0"], g["inp"], g["expected"]
    assert exp.shape == (256, out0.shape[0], 8, 8)
    for c in range(256):
        for s in range(out0.shape[0]):
            got = oracle.muladd(out0[s], inp[s], c).view(np.uint64).reshape(8, 8)
            assert np.array_equal(got, exp[c, s]), "constant 0x%02X sample %d" % (c, s)


def test_gf_tables(oracle):
    for a in range(256):
        for b in (0, 1, 2, 3, 0x1D, 0x80, 0xFF, a):
            assert oracle.gf_mul(a, b) == py_gf_mul(a, b)
    for a in range(1, 256):
        assert oracle.gf_div(1, a) == py_gf_inv(a)
        assert oracle.gf_mul(a, oracle.gf_div(1, a)) == 1
    # ec-galois.c: invalid operands return the field size
    assert oracle.gf_mul(256, 1) == 256
    assert oracle.gf_div(3, 0) == 256
    assert oracle.gf_exp(0, 0) == 256


def test_encode_matrix_is_reversed_vandermonde(oracle):
    for k, n in ((2, 3), (4, 6), (8, 12), (16, 20), (16, 31)):
        m = oracle.encode_matrix(k, n)
        for i in range(n):
            v = i + 1
            for j in range(k):
                e = 1
                for _ in range(k - 1 - j):
                    e = py_gf_mul(e, v)
                assert m[i, j] == e


def test_inverse_matches_survey_appendix_c(oracle):
    fx = json.load(open(os.path.join(GOLD, "survey_appendix_c.json")))
    inv = fx["inverse"]
    assert oracle.inverse_matrix([3, 4, 5, 6]).tolist() == inv["4+2 mask 0x3C rows [3,4,5,6]"]
    assert oracle.inverse_matrix([1, 2, 3, 4]).tolist() == inv["4+2 mask 0x0F rows [1,2,3,4]"]


def test_zero_census_4p2(oracle):
    fx = json.load(open(os.path.join(GOLD, "survey_appendix_c.json")))["zero_census_4p2"]
    counts = {0: 0, 1: 0, 2: 0}
    for rows in itertools.combinations(range(1, 7), 4):
        z = int((oracle.inverse_matrix(list(rows)) == 0).sum())
        counts[z] = counts.get(z, 0) + 1
    assert counts[0] == fx["with_0_zeros"]
    assert counts[1] == fx["with_1_zero"]
    assert counts[2] == fx["with_2_zeros"]


@pytest.mark.parametrize("k,n", [(2, 3), (4, 6), (8, 12), (16, 20)])
def test_inverse_matches_gauss_jordan(oracle, k, n):
    rng = np.random.default_rng(k * 100 + n)
    E = oracle.encode_matrix(k, n)
    combos = list(itertools.combinations(range(n), k))
    for idx in rng.choice(len(combos), size=min(20, len(combos)), replace=False):
        rows = combos[idx]
        want = py_inverse([list(map(int, E[r])) for r in rows])
        got = oracle.inverse_matrix([r + 1 for r in rows]).tolist()
        assert got == want


def gf_matvec_chunks(coef_row, chunks):
    """Reference-independent symbol-level combination of 512-B chunks."""
    out = np.zeros(512 * 8, dtype=np.uint8)  # 512 symbols as bytes (unpacked)
    for c, ch in zip(coef_row, chunks):
        bits = np.unpackbits(ch.reshape(8, 64), axis=1, bitorder="little")  # [plane][sym]
        sym = np.zeros(512, dtype=np.int64)
        for b in range(8):
            sym |= bits[b].astype(np.int64) << b
        prod = np.array([py_gf_mul(int(c), int(s)) for s in sym], dtype=np.int64)
        out[:512] ^= prod.astype(np.uint8)
    sym = out[:512]
    planes = np.stack([(sym >> b) & 1 for b in range(8)]).astype(np.uint8)
    return np.packbits(planes, axis=1, bitorder="little").reshape(-1)


def test_encode_symbol_level_restatement(oracle):
    """Appendix B layout: byte b*64 + s/8, bit s%8 holds bit b of symbol s."""
    k, n = 4, 6
    data = oracle.fill_xorshift(512 * k * 2)
    frags = oracle.encode(k, n, data)
    E = oracle.encode_matrix(k, n)
    for t in range(2):
        chunks = [data[(t * k + j) * 512:(t * k + j + 1) * 512] for j in range(k)]
        for i in range(n):
            want = gf_matvec_chunks(E[i], chunks)
            assert np.array_equal(frags[i][t * 512:(t + 1) * 512], want)


@pytest.mark.parametrize("k,n", [(2, 1 + 2), (3, 4), (4, 6), (8, 12), (16, 20)])
def test_roundtrip_all_or_sampled_masks(oracle, k, n):
    nst = 3
    data = oracle.fill_xorshift(512 * k * nst, seed=0x1234 + k)
    frags = oracle.encode(k, n, data)
    combos = list(itertools.combinations(range(n), k))
    rng = np.random.default_rng(7)
    pick = combos if len(combos) <= 40 else [combos[i] for i in
                                              rng.choice(len(combos), 40, replace=False)]
    for rows in pick:
        out = oracle.decode(k, [r + 1 for r in rows], [frags[r] for r in rows])
        assert np.array_equal(out, data), rows


def test_mt_matches_single(oracle):
    k, n = 4, 6
    data = oracle.fill_xorshift(512 * k * 101, seed=99)
    a = oracle.encode(k, n, data)
    b = oracle.encode(k, n, data, nthreads=5)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    rows = [2, 3, 5, 6]
    d1 = oracle.decode(k, rows, [a[r - 1] for r in rows])
    d2 = oracle.decode(k, rows, [a[r - 1] for r in rows], nthreads=3)
    assert np.array_equal(d1, d2) and np.array_equal(d1, data)


def test_xorshift_known_start(oracle):
    buf = oracle.fill_xorshift(16).view(np.uint64)
    x = 0x9E3779B97F4A7C15
    want = []
    for _ in range(2):
        x ^= (x << 13) & 0xFFFFFFFFFFFFFFFF
        x ^= x >> 7
        x ^= (x << 17) & 0xFFFFFFFFFFFFFFFF
        want.append(x)
    assert buf.tolist() == want


def test_writev_merge_pinned_by_hand(oracle):
    """oracle.writev_merge against byte positions worked out by hand from
    ec_writev_prepare_buffers / ec_merge_stripe_{head,tail}_locked
    (ec-inode-write.c:1825-1908) for a 2+1 volume (stripe 1024)."""
    import numpy as np
    S = 1024
    oh = np.arange(S, dtype=np.uint32).astype(np.uint8)
    ot = (255 - np.arange(S, dtype=np.uint32)).astype(np.uint8)
    user = np.full(50, 7, np.uint8)
    v = oracle.writev_merge(2, 1000, user, oh, ot)       # spans two stripes
    assert v.size == 2048
    assert np.array_equal(v[:1000], oh[:1000])
    assert np.array_equal(v[1000:1050], user)
    assert np.array_equal(v[1050:], ot[26:])               # tail = 998 bytes
    v = oracle.writev_merge(2, 10, user, oh, ot)          # one stripe: both ends old_head
    assert v.size == S and np.array_equal(v[:10], oh[:10])
    assert np.array_equal(v[60:], oh[60:])
    v = oracle.writev_merge(2, 0, user, None, ot)         # head 0: tail from old_tail
    assert np.array_equal(v[50:], ot[50:])
    v = oracle.writev_merge(2, 10, user, None, None)      # beyond EOF: zeros
    assert v[:10].sum() == 0 and v[60:].sum() == 0
