"""N>1 path on CPU: two gloo ranks shard a disperse job by stripe range
(glusterfs_amd/dist.py, the code bench.py runs under torch.distributed.run)
and the union of their shards equals the single-process result.  The per-rank
compute is the CPU oracle (test stand-in for the GPU kernel)."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, k, n, nstripes, group, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import oracle as O
    from glusterfs_amd.dist import Group, stripe_range

    g = Group(backend="gloo")
    data = O.fill_xorshift(512 * k * nstripes)
    s0, s1 = stripe_range(g.rank, g.world, nstripes, align=group)
    mine = O.encode(k, n, data[s0 * 512 * k:s1 * 512 * k]) if s1 > s0 else \
        [np.zeros(0, np.uint8)] * n
    # gather shards (test-only collective) and compare with the full encode
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    g.dist.all_gather(sizes, torch.tensor([s1 - s0]))
    full = O.encode(k, n, data)
    ok = True
    for i in range(n):
        buf = torch.zeros(max(int(x.item()) for x in sizes) * 512, dtype=torch.uint8)
        buf[:(s1 - s0) * 512] = torch.from_numpy(mine[i])
        parts = [torch.zeros_like(buf) for _ in range(world)]
        g.dist.all_gather(parts, buf)
        cat = np.concatenate([p[:int(sz.item()) * 512].numpy() for p, sz in zip(parts, sizes)])
        ok &= np.array_equal(cat, full[i])
    elapsed = g.max(0.5 + rank)          # max-over-ranks timing
    ok = g.all_ok(ok)
    g.close()
    q.put((rank, ok, elapsed, s0, s1))


@pytest.mark.parametrize("nstripes,group", [(1000, 1), (999, 16), (7, 1)])
def test_two_rank_stripe_partition(nstripes, group):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    ps = [ctx.Process(target=_worker, args=(r, world, port, 4, 6, nstripes, group, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] for r in res)
    assert all(r[2] == 1.5 for r in res)           # max over ranks of 0.5 + rank
    assert res[0][3] == 0 and res[-1][4] == nstripes
    assert res[0][4] == res[1][3]                   # contiguous, disjoint
    if group > 1:
        assert res[0][4] % group == 0


def test_stripe_range_properties():
    from glusterfs_amd.dist import stripe_range
    for n in (0, 1, 7, 1000, 524288):
        for w in (1, 2, 3, 8):
            for al in (1, 8, 1024):
                rs = [stripe_range(r, w, n, al) for r in range(w)]
                assert rs[0][0] == 0 and rs[-1][1] == n
                for (a0, a1), (b0, b1) in zip(rs, rs[1:]):
                    assert a1 == b0 and a0 <= a1
                    assert a1 % al == 0 or a1 == n


def _strong_worker(rank, world, port, nstripes, q):
    """configs[3] strong split on CPU: each rank generates ONLY its slice of
    the one xorshift stream (synth.fill_numpy jump-ahead, the bench's
    word0 = s0 * 512 * k / 8) and encodes it with the product's CPU engine;
    the gathered fragments must equal the oracle's encode of the whole job."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "oracle")]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import oracle as O
    import glusterfs_amd as g
    from glusterfs_amd import synth
    from glusterfs_amd.dist import Group, stripe_range

    k, n = 16, 20
    grp = Group(backend="gloo")
    s0, s1 = stripe_range(grp.rank, grp.world, nstripes)
    mine = synth.fill_numpy((s1 - s0) * 512 * k, word0=s0 * 512 * k // 8)
    frags = [np.zeros((s1 - s0) * 512, np.uint8) for _ in range(n)]
    with g.ECMatrixList(k, n, gen="none") as L:
        L.encode_batch(s1 - s0, mine, frags)
    parts = grp.gather([f.tobytes() for f in frags])
    ok = True
    if grp.rank == 0:
        full = O.encode(k, n, O.fill_xorshift(nstripes * 512 * k))
        for i in range(n):
            cat = b"".join(p[i] for p in parts)
            ok &= cat == full[i].tobytes()
    ok = grp.all_ok(ok)
    grp.close()
    q.put((rank, ok, s0, s1))


@pytest.mark.parametrize("world", [2, 4])
def test_two_rank_strong_job(world):
    """2 ranks, and 4 (a rehearsal of more ranks than the CI's gloo pair;
    the 8-GPU run is the driver's)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    nst = 1001
    ps = [ctx.Process(target=_strong_worker, args=(r, world, port, nst, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] for r in res)
    assert res[0][2] == 0 and res[-1][3] == nst
    assert all(a[3] == b[2] for a, b in zip(res, res[1:]))     # contiguous, disjoint


def test_bind_to_node(tmp_path):
    """bench.py's rank placement: the rank keeps the CPUs of its GPU's NUMA
    node that it may use (sysfs cpulist format), and nothing changes for an
    unknown node or a node without usable CPUs."""
    from glusterfs_amd.dist import bind_to_node, parse_cpulist
    assert parse_cpulist("0-3,8,10-11\n") == {0, 1, 2, 3, 8, 10, 11}
    aff = set(os.sched_getaffinity(0))
    try:
        assert bind_to_node(-1) == aff
        node = tmp_path / "node0"
        node.mkdir()
        pick = sorted(aff)[:1]
        (node / "cpulist").write_text("%d\n" % pick[0])
        assert bind_to_node(0, sysfs=str(tmp_path)) == set(pick)
        assert set(os.sched_getaffinity(0)) == set(pick)
        (node / "cpulist").write_text("100000\n")            # no usable CPU: unchanged
        assert bind_to_node(0, sysfs=str(tmp_path)) == set(pick)
    finally:
        os.sched_setaffinity(0, aff)


def _eight_rank_worker(rank, world, port, q):
    """One of 8 gloo ranks of configs[3]'s strong job: the
    rank's placement as bench.py's bind_rank makes it, with the GPU pool's
    16-CPU quota split 8 ways, then its 1 GiB slice of the 8 GiB job --
    generated alone by jump-ahead, encoded by the product's CPU engine -- and
    its input and 20 fragments against the slice's SHA-256 fixture."""
    import hashlib
    import importlib.util
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root]
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), EC_MI355X_QUIET="1")
    os.environ.pop("EC_COPY_THREADS", None)
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    import glusterfs_amd as g
    from glusterfs_amd import synth
    from glusterfs_amd.dist import Group, stripe_range

    # the pool's quota (16 CPUs for all ranks of a node), whatever this host has
    real = bench.host_cpus
    bench.host_cpus = lambda: dict(real(), cgroup_quota=16, threads=16)
    placement = bench.bind_rank(g, rank, world)
    copy_env = os.environ.get("EC_COPY_THREADS")
    fx = json.load(open(os.path.join(root, "tests", "golden", "fullsize_sha256.json")))
    case = fx["cases"]["16+4_8GiBjob_N%d_r%d" % (world, rank)]
    k, n = 16, 20
    grp = Group(backend="gloo")
    s0, s1 = stripe_range(grp.rank, grp.world, bench.STRONG_STRIPES)
    ok = (s1 - s0) * 512 * k == case["bytes"]
    data = synth.fill_numpy((s1 - s0) * 512 * k, word0=s0 * 512 * k // 8)
    ok &= hashlib.sha256(data).hexdigest() == case["data"]
    frags = [np.empty((s1 - s0) * 512, np.uint8) for _ in range(n)]
    with g.ECMatrixList(k, n, gen="avx") as L:
        L.encode_batch(s1 - s0, data, frags)
    del data
    ok &= [hashlib.sha256(f).hexdigest() for f in frags] == case["frags"]
    del frags
    ok_all = grp.all_ok(ok)
    grp.close()
    q.put((rank, ok, ok_all, s0, s1, copy_env, placement["copy_threads"]))


def test_eight_rank_strong_job_fixtures():
    """N = 8 rehearsed on the CPU before the driver's first 8-GPU run: eight
    gloo ranks, the 8 GiB configs[3] job cut into eight 1 GiB slices, each
    slice's input and fragments against its own fixture; bind_rank gives
    every rank 16 / 8 = 2 copy threads."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 8
    ps = [ctx.Process(target=_eight_rank_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=600) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(r[1] for r in res), [r[:2] for r in res]       # each slice vs its fixture
    assert all(r[2] for r in res)                              # and the all-ranks flag
    assert res[0][3] == 0 and res[-1][4] == 1 << 20
    assert all(a[4] == b[3] for a, b in zip(res, res[1:]))     # contiguous, disjoint
    assert all(r[5] == "2" for r in res), [r[5] for r in res]  # 16 CPUs / 8 ranks
    assert all(r[6] == 2 for r in res), [r[6] for r in res]    # as the library applies it
