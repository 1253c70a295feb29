"""On-disk format guard: the library's
trusted.ec.config helpers against the CPU restatement of the reference
(oracle/config.py: ec-helpers.c:298-380, ec-common.c:1151-1195).  No GPU."""
import errno
import itertools

import pytest

import config as R  # oracle/config.py -- test infrastructure


@pytest.fixture(scope="module")
def m():
    import glusterfs_amd.ec_method as m
    return m


def mk(m, d):
    c = m.Config()
    for k, v in d.items():
        setattr(c, k, v)
    return c


def test_golden_4p2_value(m):
    """A 4+2 volume stores 0x0000080602000200 (bit layout of ec-helpers.c:313-318)."""
    v = m.config_pack(m.config_fill(6, 2))
    assert v == bytes.fromhex("0000080602000200")
    assert v == R.pack(R.fill(6, 2))


@pytest.mark.parametrize("k,r", [(2, 1), (4, 2), (8, 4), (16, 4), (16, 15), (10, 3)])
def test_fill_pack_unpack_check_round_trip(m, k, r):
    c = m.config_fill(k + r, r)
    assert c.astuple() == tuple(R.fill(k + r, r).values())
    u = m.config_unpack(m.config_pack(c))
    assert u.astuple() == c.astuple()
    assert m.config_check(k + r, r, u) == 0
    # the same fragments opened by a volume of another geometry are refused;
    # the reference calls that "unsupported" when 4096 chunk bits divide by
    # 8 x data bricks and "corrupted" otherwise (10+3: 4096 % 80 != 0)
    want = -errno.ENOTSUP if 4096 % (8 * k) == 0 else -errno.EINVAL
    assert R.check(k + r + 1, r, R.fill(k + r, r)) == (
        "unsupported" if want == -errno.ENOTSUP else "corrupted")
    assert m.config_check(k + r + 1, r, u) == want


def test_unpack_errors(m):
    with pytest.raises(OSError) as e:
        m.config_unpack(bytes(8))
    assert e.value.errno == errno.ENODATA          # zero = absent xattr
    for bad in (bytes(7), bytes(9), bytes.fromhex("0100080602000200")):
        with pytest.raises(OSError) as e:
            m.config_unpack(bad)
        assert e.value.errno == errno.EINVAL
    c = m.config_fill(6, 2)
    c.version = 1
    with pytest.raises(OSError) as e:
        m.config_pack(c)
    assert e.value.errno == errno.EINVAL


def test_check_matches_reference_over_grid(m):
    """ec_config_check's three outcomes over a grid of every field,
    including corrupt values (word size 0 / not a power of two, chunk bits
    not divisible, redundancy 0 or >= half the bricks)."""
    n = 0
    for version, alg, w, bricks, red, chunk in itertools.product(
            (0,), (0, 1), (0, 1, 3, 8, 16), (0, 3, 6, 7, 12, 20, 31, 255),
            (0, 1, 2, 3, 4, 15, 255), (0, 256, 512, 513, 4096, 0xFFFFFF)):
        d = dict(version=version, algorithm=alg, gf_word_size=w, bricks=bricks,
                 redundancy=red, chunk_size=chunk)
        for nodes, rr in ((6, 2), (12, 4)):
            want = R.check(nodes, rr, d)
            got = m.config_check(nodes, rr, mk(m, d))
            assert got == {True: 0, "corrupted": -errno.EINVAL,
                           "unsupported": -errno.ENOTSUP}[want], (d, nodes, rr)
            n += 1
        # pack / unpack agree with the restatement on every value
        v = R.pack(d)
        assert m.config_pack(mk(m, d)) == v
        want = R.unpack(v)
        if isinstance(want, int):
            with pytest.raises(OSError) as e:
                m.config_unpack(v)
            assert -e.value.errno == want
        else:
            assert m.config_unpack(v).astuple() == tuple(want.values())
    assert n > 5000


@pytest.mark.gpu
@pytest.mark.parametrize("k,r", [(4, 2), (8, 4), (16, 4)])
def test_gpu_written_bricks_read_by_cpu_client(m, oracle, k, r):
    """Fragments coded on MI355X plus the config xattr the xlator stores with
    them: a CPU client (the oracle restatement of the reference) accepts the
    config and decodes the fragments from every k-subset we try."""
    import numpy as np
    import glusterfs_amd as g
    n, nst = k + r, 257
    data = np.random.default_rng(k).integers(0, 256, 512 * k * nst, dtype=np.uint8)
    frags = [np.zeros(512 * nst, np.uint8) for _ in range(n)]
    with g.ECMatrixList(k, n) as L:
        L.encode_batch(nst, data, frags)
    xattr = m.config_pack(m.config_fill(n, r))
    cfg = R.unpack(xattr)
    assert R.check(n, r, cfg) is True
    rng = np.random.default_rng(1)
    for _ in range(4):
        rows = sorted(int(b) + 1 for b in rng.choice(n, k, replace=False))
        assert np.array_equal(oracle.decode(k, rows, [frags[x - 1] for x in rows]), data)
