"""GPU parity of the A/B settings that remain in the library (r03 pruned
the losing instantiations: DESIGN.md 3.4).

EC_MI355X_ENC=0 runs every device encode through the register-resident
ec_encode_vander (the kernel 2+1 uses by default);
EC_MI355X_PATCACHE=0 uploads the device pattern table of every mixed call
instead of caching it; EC_MI355X_LDSNT=1 stages these small calls with the
non-temporal LDS-DMA loads that the library uses above 256 MiB of input;
EC_MI355X_ZCDB=0 runs host-buffer combines (k <= 8) through the one tile per
block zero-copy kernel instead of the persistent double-buffered one (the
default since r04; =1 forces it), each with host encode, decode, heal and
mixed calls; EC_ZC_TPB (fixed tiles per block) and EC_ZC_INFLIGHT_KB (input
bytes in flight per round of tiles) size the persistent zero-copy grid;
EC_MI355X_ZCENC16=0 keeps 16+4 host-buffer encodes of >= 2048 stripes on the
register-resident ec_encode_vander_zc instead of the combine with the encode
matrix as its pattern (r06).
(r06 retired the measured-negative knobs EC_MI355X_CHUNK_MB,
EC_MI355X_TILE_PERM and EC_HELPER_SPIN_US from the product: the XCD tile
order is now a compile-time choice of the >= 4 GiB 16+4 encoder, covered by
test_gpu_fullsize.py's 4 GiB slices of the 8 GiB job.)  Each runs here in its own process through the C ABI, bit-exact against the
oracle on device-resident encode, full / partial decode (ragged tiles
included) and mixed decode.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import itertools, sys
sys.path.insert(0, "oracle")
import numpy as np, torch
import glusterfs_amd as g
import oracle as O           # the checker

rng = np.random.default_rng(7)
def rb(n):
    return rng.integers(0, 256, n, dtype=np.uint8)
def dev(a):
    return torch.from_numpy(a).cuda()

for k, n in ((4, 6), (8, 12), (16, 20)):
    allm = [sum(1 << b for b in c) for c in itertools.combinations(range(n), k)]
    pick = np.random.default_rng(k).choice(len(allm), min(24, len(allm)), replace=False)
    masks = [allm[i] for i in sorted(pick)]
    with g.ECMatrixList(k, n) as L:
        for nst in (13, 77, 1031):
            data = rb(512 * k * nst)
            want = O.encode(k, n, data)
            outs = [torch.empty(512 * nst, dtype=torch.uint8, device="cuda") for _ in range(n)]
            L.encode_batch(nst, dev(data), outs)
            for i in range(n):
                assert np.array_equal(outs[i].cpu().numpy(), want[i]), ("enc", k, n, nst, i)
            frags = [rb(512 * nst) for _ in range(n)]
            dfr = [dev(f) for f in frags]
            out = torch.empty(512 * k * nst, dtype=torch.uint8, device="cuda")
            for m in masks:
                rows = O.mask_rows(m)
                out.fill_(0xA5)
                L.decode_batch(nst, m, rows, [dfr[r - 1] for r in rows], out)
                exp = O.decode(k, rows, [frags[r - 1] for r in rows])
                assert np.array_equal(out.cpu().numpy(), exp), ("dec", k, n, nst, hex(m))
        group, ng = 16, 12
        nst = group * ng
        frags = [rb(512 * nst) for _ in range(n)]
        ms = masks[:6]
        ids = rng.integers(0, len(ms), ng).astype(np.uint8)
        out = torch.empty(512 * k * nst, dtype=torch.uint8, device="cuda")
        L.decode_mixed_device(0, None, nst, group, dev(ids), ms, [dev(f) for f in frags], out)
        g.sync_device(0)
        got = out.cpu().numpy()
        span = 512 * group
        for gi in range(ng):
            rows = O.mask_rows(ms[ids[gi]])
            exp = O.decode(k, rows, [frags[r - 1][gi * span:(gi + 1) * span] for r in rows])
            assert np.array_equal(got[gi * span * k:(gi + 1) * span * k], exp), ("mixed", k, gi)
        # host buffers (EC_GPU_ALWAYS=1: the zero-copy combine over staged
        # pinned slots), several tiles per block of the persistent kernel
        for nst in (5, 1031, 4100):
            hdata = rb(512 * k * nst)
            hf = [np.empty(512 * nst, np.uint8) for _ in range(n)]
            L.encode_batch(nst, hdata, hf)
            wantf = O.encode(k, n, hdata)
            for i in range(n):
                assert np.array_equal(hf[i], wantf[i]), ("host enc", k, n, nst, i)
            frags = [rb(512 * nst) for _ in range(n)]
            out = np.empty(512 * k * nst, np.uint8)
            for m in masks[:4]:
                rows = O.mask_rows(m)
                L.decode_batch(nst, m, rows, [frags[r - 1] for r in rows], out)
                exp = O.decode(k, rows, [frags[r - 1] for r in rows])
                assert np.array_equal(out, exp), ("host dec", k, n, nst, hex(m))
            # host heal (fragment-major output rows) and a host mixed decode
            m = masks[1]
            rows = O.mask_rows(m)
            tgt = [b for b in range(n) if not (m >> b) & 1][:2]
            tmask = sum(1 << b for b in tgt)
            hout = [np.empty(512 * nst, np.uint8) for _ in tgt]
            L.heal(nst, m, [frags[r - 1] for r in rows], tmask, hout)
            data = O.decode(k, rows, [frags[r - 1] for r in rows])
            full = O.encode(k, n, data)
            for j, b in enumerate(tgt):
                assert np.array_equal(hout[j], full[b]), ("host heal", k, n, nst, b)
            grp = 4 if nst % 4 == 0 else 1
            gm = [masks[(i * 7) % 4] for i in range((nst + grp - 1) // grp)]
            L.decode_mixed(nst, grp, gm, frags, out)
            for gi, gmask in enumerate(gm):
                rws = O.mask_rows(gmask)
                a0, a1 = gi * grp * 512, min(nst, (gi + 1) * grp) * 512
                exp = O.decode(k, rws, [frags[r - 1][a0:a1] for r in rws])
                assert np.array_equal(out[a0 * k:a1 * k], exp), ("host mixed", k, n, nst, gi)
assert g.ec_method.stats()["cpu_fallbacks"] == 0   # every host call ran on the GPU
print("ok")
"""

KNOBS = [("EC_MI355X_ENC", "0"), ("EC_MI355X_PATCACHE", "0"), ("EC_MI355X_LDSNT", "1"),
         ("EC_MI355X_ZCDB", "0"), ("EC_MI355X_ZCDB", "1"), ("EC_ZC_TPB", "1"), ("EC_ZC_TPB", "16"),
         ("EC_ZC_INFLIGHT_KB", "64"), ("EC_MI355X_ZCENC16", "0")]


@pytest.mark.parametrize("knob,value", KNOBS, ids=["%s=%s" % kv for kv in KNOBS])
def test_ab_instantiation_bit_exact(knob, value):
    env = dict(os.environ, EC_MI355X_QUIET="1", EC_GPU_ALWAYS="1")
    env[knob] = value
    r = subprocess.run([sys.executable, "-c", SCRIPT], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=170)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr[-3000:]
