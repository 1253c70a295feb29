"""Every BASELINE.json config at its full size, on the GPU, against the
oracle's SHA-256 fixtures (tests/golden/fullsize_sha256.json, generated in the
container by tests/golden/gen_fullsize_sha.py from oracle/ec_oracle.c).

The input is the xorshift64 stream of SURVEY 8(d), generated on the device
(glusterfs_amd/synth.py: bit-exact with the oracle's sequential fill, checked
by tests/test_fixtures.py); rank r of an N-GPU job owns the r-th slice.  Each
case checks the input hash, then every fragment the library writes, then the
decoded data (= the input, whose hash is pinned) -- the reference's stripe
loops, ec-method.c:394-433, at the sizes bench.py times.

  configs[1]  4+2 1 GiB decode, masks 0x3C and 0x0F (and the encode feeding it)
  configs[2]  8+4 64K-stripe batch encode, decode 0xFF0 and 0xEB5
  configs[3]  16+4 2 GiB encode for rank 0 and rank 1 (the stream offset of a
              stripe-range partition), and rank 0 through the pinned-host
              (PCIe) path; the one 8 GiB job (1,048,576 stripes) strong-split
              over N = 2 ranks: slices 0 and 1 (4 GiB each) on this GPU
              against tests/golden/gen_strong_sha.py's per-slice fixtures
  configs[4]  self-heal: 8+4 1 GiB with 16 masks in 1024-stripe groups, 16+4
              1 GiB with 64 masks (device decode-matrix table)
"""
import hashlib
import json
import math
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 512
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _fixtures():
    with open(os.path.join(ROOT, "tests", "golden", "fullsize_sha256.json")) as f:
        return json.load(f)["cases"]


FIX = _fixtures()


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


def sha(t):
    a = t.cpu().numpy() if hasattr(t, "cpu") else t
    return hashlib.sha256(memoryview(np.ascontiguousarray(a))).hexdigest()


def _encoded(ec, torch, case, rank=0):
    """The fixture's input slice, generated on the device and encoded there;
    input and fragments checked against the fixture."""
    from glusterfs_amd import synth
    fx = FIX["%s_r%d" % (case, rank)]
    k, n, S = fx["k"], fx["n"], fx["bytes"]
    nst = S // (CHUNK * k)
    data = synth.fill_device(torch, S, torch.device("cuda", 0), word0=fx["word0"])
    assert sha(data) == fx["data"], "input stream slice"
    frags = [torch.empty(nst * CHUNK, dtype=torch.uint8, device="cuda") for _ in range(n)]
    L = ec.ECMatrixList(k, n)
    L.encode_device(0, None, nst, data, frags)
    ec.sync_device(0)
    if "frags" in fx:
        for i, f in enumerate(frags):
            assert sha(f) == fx["frags"][i], "%s rank %d fragment %d" % (case, rank, i)
    return L, data, frags, nst, k, n


def _decode_checks(ec, torch, L, data, frags, nst, k, masks):
    out = torch.empty_like(data)
    for m in masks:
        rows = ec.mask_rows(m)
        out.fill_(0xA5)
        L.decode_device(0, None, nst, m, [frags[r - 1] for r in rows], out)
        ec.sync_device(0)
        assert bool(torch.equal(out, data)), "decode mask %#x" % m
    del out


def test_config1_4p2_1gib_decode(ec, torch_cuda):
    """configs[1]: 4+2, 1 GiB, two fragments missing (bricks 0+1, 4+5)."""
    L, data, frags, nst, k, n = _encoded(ec, torch_cuda, "4+2_1GiB")
    with L:
        _decode_checks(ec, torch_cuda, L, data, frags, nst, k, [0x3C, 0x0F])


def test_config2_8p4_64k_stripes(ec, torch_cuda):
    """configs[2]: 8+4, one 65,536-stripe batch: encode, decode 0xFF0 / 0xEB5."""
    L, data, frags, nst, k, n = _encoded(ec, torch_cuda, "8+4_64Kstripes")
    assert nst == 65536
    with L:
        _decode_checks(ec, torch_cuda, L, data, frags, nst, k, [0xFF0, 0xEB5])


@pytest.mark.parametrize("rank", [0, 1])
def test_config3_16p4_2gib_rank_slices(ec, torch_cuda, rank):
    """configs[3]: 16+4, 2 GiB per GPU; rank 1's slice starts 2 GiB into the
    stream, so the fixture also pins the partition offset."""
    L, data, frags, nst, k, n = _encoded(ec, torch_cuda, "16+4_2GiB", rank)
    with L:
        pass
    del data, frags
    torch_cuda.cuda.empty_cache()


@pytest.mark.parametrize("rank", [0, 1])
def test_config3_16p4_8gib_job_strong_n2_slices(ec, torch_cuda, rank):
    """configs[3] as one fixed job (strong scaling, bench.py strong_job): the
    1,048,576-stripe 16+4 job cut by dist.stripe_range into two 4 GiB slices;
    each rank's slice input and its 20 fragment slices against the fixture
    (its stream offset is slice 1's start)."""
    from glusterfs_amd import dist
    fx = FIX["16+4_8GiBjob_N2_r%d" % rank]
    s0, s1 = dist.stripe_range(rank, 2, fx["job_stripes"])
    assert (s1 - s0) * CHUNK * fx["k"] == fx["bytes"]
    assert s0 * CHUNK * fx["k"] // 8 == fx["word0"]
    L, data, frags, nst, k, n = _encoded(ec, torch_cuda, "16+4_8GiBjob_N2", rank)
    with L:
        pass
    del data, frags
    torch_cuda.cuda.empty_cache()


def test_config3_16p4_2gib_pinned_host(ec, torch_cuda):
    """configs[3] through the PCIe path: pinned host input and fragments
    (ec_method_host_alloc), coded by the library's async H2D / kernel / D2H
    pipeline (ec_method_encode_batch on host buffers)."""
    from glusterfs_amd import synth
    fx = FIX["16+4_2GiB_r0"]
    k, n, S = fx["k"], fx["n"], fx["bytes"]
    nst = S // (CHUNK * k)
    din = ec.ec_method.PinnedArray(S)
    frs = [ec.ec_method.PinnedArray(nst * CHUNK) for _ in range(n)]
    try:
        din.array[:] = synth.fill_numpy(S)
        assert sha(din.array) == fx["data"]
        with ec.ECMatrixList(k, n) as L:
            L.encode_batch(nst, din.ptr, [f.ptr for f in frs])
        for i, f in enumerate(frs):
            assert sha(f.array) == fx["frags"][i], "fragment %d" % i
    finally:
        for p in [din] + frs:
            p.free()


def _mixed(ec, torch, case, nmasks, group, seed):
    """configs[4]: every `group`-stripe group decoded from its own k-of-n
    brick set, drawn (seeded) from `nmasks` masks; as bench.py run_mixed."""
    L, data, frags, nst, k, n = _encoded(ec, torch, case)
    rnd = random.Random(seed)
    nmasks = min(nmasks, math.comb(n, k))
    masks = []
    while len(masks) < nmasks:
        m = sum(1 << b for b in rnd.sample(range(n), k))
        if m not in masks:
            masks.append(m)
    ngroups = (nst + group - 1) // group
    gp = torch.tensor([rnd.randrange(nmasks) for _ in range(ngroups)], dtype=torch.uint8,
                      device="cuda")
    out = torch.empty_like(data)
    with L:
        L.decode_mixed_device(0, None, nst, group, gp, masks, frags, out)
        ec.sync_device(0)
    assert bool(torch.equal(out, data))


def test_config4_selfheal_8p4_16masks(ec, torch_cuda):
    _mixed(ec, torch_cuda, "8+4_1GiB", 16, 1024, 17)


def test_config4_selfheal_16p4_64masks(ec, torch_cuda):
    _mixed(ec, torch_cuda, "16+4_1GiB", 64, 1024, 21)
