"""Guards on the device paths:

* inputs at any byte alignment: the tile encoders and every combine stage
  their inputs by LDS-DMA in 16-byte pieces, which honours any source
  address (r03, tools/kbench/ldsdma_align.hip), so a device input at an odd
  offset (a torch slice) is read in place -- bit-exact with the oracle;
* the per-thread host-page cache of the pointer classification
  (ec_device.hip ecd_ptr_device) expires, so a recycled address is
  re-queried: counted with EC_MI355X_DEBUG=1 in a child process;
* the device decode-matrix table cache evicts entries whose readers ran on
  several streams (per-stream reader events, no device-wide sync).
"""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CHUNK = 512
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rnd(n, seed):
    return np.random.default_rng(seed).integers(0, 256, size=n, dtype=np.uint8)


@pytest.fixture(scope="module")
def ec():
    import glusterfs_amd as g
    if g.device_count() < 1:
        pytest.fail("no MI355X visible")
    return g


@pytest.mark.parametrize("off", [1, 3, 4, 8, 13])
@pytest.mark.parametrize("k,n,nst", [(4, 6, 1000), (8, 12, (1 << 17) + 5), (16, 20, 777),
                                     (5, 7, 300)])
def test_encode_device_misaligned_input(ec, oracle, k, n, nst, off):
    import torch
    data = rnd(CHUNK * k * nst, seed=k * 10 + off)
    want = oracle.encode(k, n, data, nthreads=8)
    raw = torch.empty(data.size + 16, dtype=torch.uint8, device="cuda")
    din = raw[off:off + data.size]
    din.copy_(torch.from_numpy(data))
    assert din.data_ptr() % 16 == off
    outs = [torch.empty(CHUNK * nst, dtype=torch.uint8, device="cuda") for _ in range(n)]
    with ec.ECMatrixList(k, n) as L:
        L.encode_batch(nst, din, outs)
    for i in range(n):
        assert np.array_equal(outs[i].cpu().numpy(), want[i]), "fragment %d" % i


@pytest.mark.parametrize("off", [1, 4, 8])
@pytest.mark.parametrize("k,n,mask", [(4, 6, 0x3C), (8, 12, 0xEB5), (16, 20, 0xFFFF0)])
def test_decode_device_misaligned_fragments(ec, oracle, k, n, mask, off):
    """Every fragment at its own misalignment (off, off+1, ...) and the
    decoded output at an odd offset as well."""
    import torch
    nst = 333
    frags = [rnd(CHUNK * nst, seed=50 + i) for i in range(n)]
    rows = oracle.mask_rows(mask)
    want = oracle.decode(k, rows, [frags[r - 1] for r in rows])
    dfr = []
    for i, f in enumerate(frags):
        o = (off + i) % 16
        raw = torch.empty(f.size + 16, dtype=torch.uint8, device="cuda")
        t = raw[o:o + f.size]
        t.copy_(torch.from_numpy(f))
        dfr.append(t)
    rawo = torch.empty(CHUNK * k * nst + 16, dtype=torch.uint8, device="cuda")
    out = rawo[off:off + CHUNK * k * nst]
    with ec.ECMatrixList(k, n) as L:
        L.decode_batch(nst, mask, rows, [dfr[r - 1] for r in rows], out)
    assert np.array_equal(out.cpu().numpy(), want)


def test_heal_and_mixed_device_misaligned(ec, oracle):
    import torch
    k, n, nst, group = 8, 12, 4096, 512
    data = rnd(CHUNK * k * nst, seed=41)
    frags = oracle.encode(k, n, data)
    dfr = []
    for i, f in enumerate(frags):
        raw = torch.empty(f.size + 16, dtype=torch.uint8, device="cuda")
        t = raw[3:3 + f.size]
        t.copy_(torch.from_numpy(f))
        dfr.append(t)
    masks = [0xFF0, 0xEB5, 0x0FF, 0xF0F]
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


_CHILD = textwrap.dedent("""
    import sys, time
    sys.path[:0] = [%r]
    import numpy as np
    import glusterfs_amd as g
    k, n, nst = 4, 6, 64
    data = np.random.default_rng(1).integers(0, 256, 512 * k * nst, dtype=np.uint8)
    frags = [np.zeros(512 * nst, np.uint8) for _ in range(n)]
    with g.ECMatrixList(k, n) as L:
        for _ in range(50):                  # within the TTL: one query per buffer page
            L.encode_batch(nst, data, frags)
        time.sleep(0.25)                     # past the TTL: queried again
        for _ in range(50):
            L.encode_batch(nst, data, frags)
""")


def _queries(env_extra):
    env = dict(os.environ, EC_MI355X_DEBUG="1", EC_GPU_ALWAYS="0", EC_CPU_BELOW_KB="100000")
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", _CHILD % ROOT], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stderr.splitlines() if "pointer queries" in l][-1]
    return int(line.split(":")[1].split()[0])


def test_host_page_cache_expires():
    """7 host buffers (input + 6 fragments) per call, 100 CPU-routed calls in
    two bursts 250 ms apart: with the default 20 ms lifetime the pages are
    queried once per burst (not per call); with EC_HOSTPAGE_MS=0 every call
    queries; with a lifetime longer than the run, once in all."""
    per_call = 7
    q_default = _queries({})
    q_never = _queries({"EC_HOSTPAGE_MS": "0"})
    q_long = _queries({"EC_HOSTPAGE_MS": "10000"})
    # (two buffers whose pages share a cache slot evict each other on every
    # call, so the bounds leave room for such a collision)
    assert q_never >= 100 * per_call, q_never
    assert q_long < q_default < q_never // 2, (q_default, q_long, q_never)


def test_pattern_table_eviction_across_streams(ec, oracle):
    """More live mask sets (20) than cache entries (16), each decoded on
    three streams in turn, so evicted entries had readers on several
    streams; every group checked against the oracle."""
    import torch
    k, n, group, per = 16, 20, 8, 12
    nst = group * per
    frags = [rnd(CHUNK * nst, seed=700 + f) for f in range(n)]
    dfr = [torch.from_numpy(f).cuda() for f in frags]
    gp = torch.arange(per, dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(9)
    sets = []
    for _ in range(20):
        s = []
        while len(s) < per:
            m = sum(1 << int(b) for b in rng.choice(n, k, replace=False))
            if m not in s:
                s.append(m)
        sets.append(s)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.empty(CHUNK * k * nst, dtype=torch.uint8, device="cuda") for _ in sets]
    with ec.ECMatrixList(k, n) as L:
        for rep in range(2):
            for i, masks in enumerate(sets):
                st = streams[(i + rep) % 3]
                L.decode_mixed_device(0, st.cuda_stream, nst, group, gp, masks, dfr, outs[i])
        torch.cuda.synchronize()
    for i, masks in enumerate(sets):
        got = outs[i].cpu().numpy()
        for g, m in enumerate(masks):
            rows = oracle.mask_rows(m)
            want = oracle.decode(k, rows, [frags[r - 1][g * group * CHUNK:(g + 1) * group * CHUNK]
                                           for r in rows])
            assert np.array_equal(got[g * group * CHUNK * k:(g + 1) * group * CHUNK * k], want)
