"""GPU parity of partial-stripe writes:
ec_method_writev_encode / _device against the oracle's restatement of the
reference's read-modify-write (oracle.writev_merge: ec-inode-write.c:
1825-1908, 1987-2085) followed by the oracle encode.  Bit-exact.

Host buffers merge in the staging copy; device buffers go through the
fused kernel (edge stripes gathered, interior read in place with
realigned loads) or, for geometries without a compile-time encoder, a
device-side gather + the generic encoder."""
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


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


def cases(S):
    """(head, user bytes, old_head?, old_tail?) covering the merge rules."""
    return [
        (0, S, True, True),            # aligned full stripe: no merge
        (0, 3 * S, False, False),
        (0, S - 1, True, True),        # one stripe, tail from old (head == 0)
        (0, S - 1, False, True),
        (1, 1, True, True),            # one stripe, both ends from old_head
        (7, S - 7, True, False),
        (5, 9, False, True),           # one stripe, old_tail only
        (3, 9, False, False),          # beyond EOF: zeros
        (S - 1, 2, True, True),        # two stripes, 1 byte each side
        (100, 5 * S + 33, True, True),
        (100, 5 * S + 33, False, True),
        (S // 2, 7 * S, True, False),
        (0, 3 * S + 1, True, True),
        (333, 40 * S + 4095, True, True),
    ]


GEOMS = [(4, 6), (8, 12), (16, 20), (5, 7), (2, 3)]


@pytest.mark.parametrize("k,n", GEOMS)
@pytest.mark.parametrize("split", [False, True])
def test_writev_host_matches_oracle(ec, oracle, k, n, split):
    S = CHUNK * k
    with ec.ECMatrixList(k, n) as L:
        for ci, (head, us, oh, ot) in enumerate(cases(S)):
            base = rnd(us + 16, seed=ci)
            user = base[ci % 13:ci % 13 + us]          # arbitrary alignment
            old_head = rnd(S, seed=100 + ci) if oh else None
            old_tail = rnd(S, seed=200 + ci) if ot else None
            v = oracle.writev_merge(k, head, user, old_head, old_tail)
            want = oracle.encode(k, n, v)
            nst = v.size // S
            out = [np.full(CHUNK * nst, 0xA5, np.uint8) for _ in range(n)]
            if split and us >= 3:                       # a writev iovec list
                a, b = us // 3, 2 * us // 3 + 1
                L.writev_encode(head, [user[:a], user[a:b], user[b:]], old_head, old_tail, out)
            else:
                L.writev_encode(head, user, old_head, old_tail, out)
            for i in range(n):
                assert np.array_equal(out[i], want[i]), (ci, head, us, "fragment", i)


@pytest.mark.parametrize("k,n", GEOMS)
def test_writev_device_matches_oracle(ec, oracle, torch_cuda, k, n):
    torch = torch_cuda
    S = CHUNK * k
    with ec.ECMatrixList(k, n) as L:
        for ci, (head, us, oh, ot) in enumerate(cases(S)):
            mis = (ci * 5) % 16
            base = rnd(us + 32, seed=ci)
            user_h = base[mis:mis + us]
            dbase = torch.from_numpy(base).cuda()
            duser = dbase[mis:mis + us]                  # odd device address
            old_head = rnd(S, seed=100 + ci) if oh else None
            old_tail = rnd(S, seed=200 + ci) if ot else None
            dh = torch.from_numpy(old_head).cuda() if oh else None
            dt = torch.from_numpy(old_tail).cuda() if ot else None
            v = oracle.writev_merge(k, head, user_h, old_head, old_tail)
            want = oracle.encode(k, n, v)
            nst = v.size // S
            out = [torch.full((CHUNK * nst,), 0xA5, dtype=torch.uint8, device="cuda")
                   for _ in range(n)]
            torch.cuda.synchronize()
            L.writev_encode_device(0, None, head, us, duser, dh, dt, out)
            torch.cuda.synchronize()
            for i in range(n):
                assert np.array_equal(out[i].cpu().numpy(), want[i]), (ci, head, us, mis, i)


@pytest.mark.parametrize("k,n", [(4, 6), (8, 12), (16, 20)])
def test_writev_device_every_byte_shift(ec, oracle, torch_cuda, k, n):
    """The interior's address modulo 16 takes every value (r05: a byte-
    misaligned interior is staged from dword-aligned loads, shifted by the
    byte offset, with the next piece's first dword taken from the
    neighbouring lane -- 16-lane DPP rows, stripe ends and the wave's last
    lane load their own), over 11 stripes (several 4-stripe tiles)."""
    torch = torch_cuda
    S = CHUNK * k
    with ec.ECMatrixList(k, n) as L:
        for shift in range(16):
            head = 700 + 37 * shift
            us = 10 * S - head + 333
            mis = (shift + head) % 16          # (user - head) % 16 == shift
            base = rnd(us + 32, seed=1000 + shift)
            user_h = base[mis:mis + us]
            dbase = torch.from_numpy(base).cuda()
            duser = dbase[mis:mis + us]
            assert (duser.data_ptr() - head) % 16 == shift
            old_head, old_tail = rnd(S, seed=2000 + shift), rnd(S, seed=3000 + shift)
            dh, dt = torch.from_numpy(old_head).cuda(), torch.from_numpy(old_tail).cuda()
            want = oracle.encode(k, n, oracle.writev_merge(k, head, user_h, old_head, old_tail))
            nst = want[0].size // CHUNK
            out = [torch.full((CHUNK * nst,), 0xA5, dtype=torch.uint8, device="cuda")
                   for _ in range(n)]
            torch.cuda.synchronize()
            L.writev_encode_device(0, None, head, us, duser, dh, dt, out)
            torch.cuda.synchronize()
            for i in range(n):
                assert np.array_equal(out[i].cpu().numpy(), want[i]), (shift, "fragment", i)


def test_writev_host_pointer_to_device_dispatch(ec, oracle, torch_cuda):
    """ec_method_writev_encode with device buffers takes the fused path."""
    torch = torch_cuda
    k, n, head, us = 4, 6, 77, 9 * CHUNK * 4 + 5
    S = CHUNK * k
    base = rnd(us + 8, seed=3)
    d = torch.from_numpy(base).cuda()
    oh = rnd(S, seed=4)
    v = oracle.writev_merge(k, head, base[3:3 + us], oh, None)
    want = oracle.encode(k, n, v)
    out = [torch.empty(v.size // k, dtype=torch.uint8, device="cuda") for _ in range(n)]
    with ec.ECMatrixList(k, n) as L:
        L.writev_encode(head, d[3:3 + us], torch.from_numpy(oh).cuda(), None, out)
    for i in range(n):
        assert np.array_equal(out[i].cpu().numpy(), want[i])


def test_writev_device_large_equals_plain_encode(ec, torch_cuda):
    """256 MiB write at an odd offset and odd address: the fused kernel equals
    the plain encoder on the materialised padded buffer (size-independent
    property; both are bit-exact elsewhere)."""
    torch = torch_cuda
    k, n = 4, 6
    S = CHUNK * k
    head, us = 1234, (256 << 20) + 777
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    base = torch.randint(0, 256, (us + 64,), dtype=torch.uint8, device="cuda", generator=g)
    user = base[13:13 + us]
    oh = torch.randint(0, 256, (S,), dtype=torch.uint8, device="cuda", generator=g)
    ot = torch.randint(0, 256, (S,), dtype=torch.uint8, device="cuda", generator=g)
    size = (head + us + S - 1) // S * S
    tail = size - head - us
    v = torch.cat([oh[:head], user, ot[S - tail:]])
    nst = size // S
    a = [torch.empty(CHUNK * nst, dtype=torch.uint8, device="cuda") for _ in range(n)]
    b = [torch.empty_like(x) for x in a]
    torch.cuda.synchronize()          # inputs made on torch's stream
    with ec.ECMatrixList(k, n) as L:
        L.writev_encode_device(0, None, head, us, user, oh, ot, a)
        L.encode_device(0, None, nst, v, b)
        torch.cuda.synchronize()
    for i in range(n):
        assert torch.equal(a[i], b[i]), i


def test_writev_errors(ec):
    import errno
    k, n = 4, 6
    with ec.ECMatrixList(k, n) as L:
        out = [np.zeros(CHUNK, np.uint8) for _ in range(n)]
        with pytest.raises(OSError) as e:
            L.writev_encode(CHUNK * k, np.zeros(4, np.uint8), None, None, out)  # head >= stripe
        assert e.value.errno == errno.EINVAL
        L.writev_encode(5, np.zeros(0, np.uint8), None, None, out)          # empty: no-op
