"""Synthetic input of SURVEY.md 8(d): xorshift64 (13, 7, 17), seed
0x9E3779B97F4A7C15, little-endian u64 words -- word i of the stream is the
generator state after i + 1 steps (the survey probe's fill, restated by
oracle/ec_oracle.c or_fill_xorshift for the fixtures).

The step is linear over GF(2)^64, so the stream can be entered at any word by
a 64x64 bit-matrix power (jump-ahead).  That lets every rank of an N-GPU job
generate its own stripe range of one global stream on its GPU, and lets the
GPU generate 1-2 GiB in parallel: the range is cut into blocks of L words,
each block's start state is computed on the host by matrix powers, and the
blocks then step in lock-step on the device (torch int64 ops).  Benchmark
data generation only; nothing here is on the coding path.
"""
import numpy as np

SEED = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1


def _step(x):
    x ^= (x << 13) & M64
    x ^= x >> 7
    x ^= (x << 17) & M64
    return x


def _matrix():
    """The step as 64 column images: column b = step(1 << b)."""
    return [_step(1 << b) for b in range(64)]


def _apply(cols, x):
    r = 0
    b = 0
    while x:
        if x & 1:
            r ^= cols[b]
        x >>= 1
        b += 1
    return r


def _mul(a, b):
    """Column form of A @ B."""
    return [_apply(a, c) for c in b]


def _pow(cols, e):
    r = [1 << b for b in range(64)]
    p = cols
    while e:
        if e & 1:
            r = _mul(p, r)
        p = _mul(p, p)
        e >>= 1
    return r


def _apply_np(cols, v):
    """Apply a column-form matrix to every element of a uint64 array."""
    out = np.zeros_like(v)
    for b in range(64):
        bit = (v >> np.uint64(b)) & np.uint64(1)
        out ^= bit * np.uint64(cols[b])
    return out


def block_states(word0, nblocks, block_words, seed=SEED):
    """State before word word0 + j * block_words, j < nblocks (uint64)."""
    m = _matrix()
    st = np.empty(nblocks, dtype=np.uint64)
    st[0] = _apply(_pow(m, word0), seed)
    p = _pow(m, block_words)
    done = 1
    while done < nblocks:
        take = min(done, nblocks - done)
        st[done:done + take] = _apply_np(p, st[:take])
        p = _mul(p, p)
        done += take
    return st


def fill_numpy(nbytes, seed=SEED, word0=0):
    """Host fill of words [word0, word0 + nbytes/8) of the stream."""
    assert nbytes % 8 == 0
    n = nbytes // 8
    L = 1024
    nb = (n + L - 1) // L
    st = block_states(word0, nb, L, seed)
    out = np.empty((L, nb), dtype=np.uint64)
    s = st.copy()
    for j in range(L):
        s ^= s << np.uint64(13)
        s ^= s >> np.uint64(7)
        s ^= s << np.uint64(17)
        out[j] = s
    return np.ascontiguousarray(out.T).reshape(-1)[:n].view(np.uint8)


def fill_device(torch, nbytes, device, seed=SEED, word0=0):
    """Device fill (uint8 tensor) of words [word0, word0 + nbytes/8)."""
    assert nbytes % 8 == 0
    n = nbytes // 8
    L = 1024
    nb = (n + L - 1) // L
    st = block_states(word0, nb, L, seed).view(np.int64)
    s = torch.from_numpy(st.copy()).to(device)
    low57 = (1 << 57) - 1                     # logical >> 7 on int64
    out = torch.empty((L, nb), dtype=torch.int64, device=device)
    for j in range(L):
        s ^= s << 13
        s ^= (s >> 7) & low57
        s ^= s << 17
        out[j] = s
    flat = out.t().contiguous().view(-1)[:n]
    del out
    return flat.view(torch.uint8)
