"""ctypes binding of oracle/libecoracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  It wraps the plain-C restatement in oracle/ec_oracle.c (see that
file's header for the reference file:line map and how parity is pinned).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libecoracle.so")
CHUNK = 512
SEED = 0x9E3779B97F4A7C15

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
        L.or_gf_mul.argtypes = [u32, u32]
        L.or_gf_mul.restype = u32
        L.or_gf_div.argtypes = [u32, u32]
        L.or_gf_div.restype = u32
        L.or_gf_exp.argtypes = [u32, u32]
        L.or_gf_exp.restype = u32
        L.or_init.argtypes = []
        L.or_matrix_normal.argtypes = [vp, u32, vp, u32]
        L.or_matrix_inverse.argtypes = [vp, vp, u32]
        L.or_prepare.argtypes = [vp, u32]
        L.or_muladd.argtypes = [vp, vp, u32]
        L.or_encode.argtypes = [u32, u32, u64, vp, vp]
        L.or_encode.restype = ctypes.c_int
        L.or_encode_mt.argtypes = [u32, u32, u64, vp, vp, u32]
        L.or_encode_mt.restype = ctypes.c_int
        L.or_decode.argtypes = [u32, u64, vp, vp, vp]
        L.or_decode.restype = ctypes.c_int
        L.or_decode_mt.argtypes = [u32, u64, vp, vp, vp, u32]
        L.or_decode_mt.restype = ctypes.c_int
        L.or_decode_matrix.argtypes = [u32, vp, vp, vp]
        L.or_decode_matrix.restype = ctypes.c_int
        L.or_fill_xorshift.argtypes = [vp, u64, u64]
        L.or_fill_xorshift.restype = u64
        L.or_init()
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def gf_mul(a, b):
    return lib().or_gf_mul(a, b)


def gf_div(a, b):
    return lib().or_gf_div(a, b)


def gf_exp(a, b):
    return lib().or_gf_exp(a, b)


def encode_matrix(k, n):
    m = np.zeros(n * k, dtype=np.uint32)
    vals = np.arange(1, n + 1, dtype=np.uint32)
    lib().or_matrix_normal(_ptr(m), k, _ptr(vals), n)
    return m.reshape(n, k)


def inverse_matrix(rows):
    """rows: ascending brick_idx + 1 values; returns the raw k x k inverse."""
    rows = np.ascontiguousarray(rows, dtype=np.uint32)
    k = rows.size
    m = np.zeros(k * k, dtype=np.uint32)
    lib().or_matrix_inverse(_ptr(m), _ptr(rows), k)
    return m.reshape(k, k)


def prepare(values):
    v = np.ascontiguousarray(values, dtype=np.uint32).copy()
    lib().or_prepare(_ptr(v), v.size)
    return v


def muladd(out_chunk, in_chunk, c):
    """out = out * c ^ in on one 512-byte chunk (returns a new array)."""
    o = np.ascontiguousarray(out_chunk).view(np.uint8).copy()
    i = np.ascontiguousarray(in_chunk).view(np.uint8)
    assert o.nbytes == CHUNK and i.nbytes == CHUNK
    lib().or_muladd(_ptr(o), _ptr(i), c)
    return o


def fill_xorshift(size, seed=SEED):
    buf = np.empty(size, dtype=np.uint8)
    lib().or_fill_xorshift(_ptr(buf), size, seed)
    return buf


def encode(k, n, data, nthreads=1, out=None):
    """data: uint8 array, size multiple of 512*k -> list of n fragments
    (written into `out`, n preallocated arrays of size/k bytes, if given)."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    fsize = data.size // k
    if out is None:
        frags = [np.empty(fsize, dtype=np.uint8) for _ in range(n)]
    else:
        frags = list(out)
        assert len(frags) == n and all(f.size == fsize and f.dtype == np.uint8 and
                                       f.flags.c_contiguous for f in frags)
    ptrs = (ctypes.c_void_p * n)(*[f.ctypes.data for f in frags])
    if nthreads > 1:
        rc = lib().or_encode_mt(k, n, data.size, _ptr(data), ptrs, nthreads)
    else:
        rc = lib().or_encode(k, n, data.size, _ptr(data), ptrs)
    if rc != 0:
        raise ValueError("or_encode rejected k=%d n=%d size=%d" % (k, n, data.size))
    return frags


def decode(k, rows, frags, nthreads=1, out=None):
    """rows: brick_idx+1 ascending (len k); frags: the k matching fragments.
    Returns the decoded data (written into `out`, size*k bytes, if given)."""
    rows = np.ascontiguousarray(rows, dtype=np.uint32)
    frags = [np.ascontiguousarray(f, dtype=np.uint8) for f in frags]
    size = frags[0].size
    if out is None:
        out = np.empty(size * k, dtype=np.uint8)
    assert out.size == size * k and out.dtype == np.uint8 and out.flags.c_contiguous
    ptrs = (ctypes.c_void_p * k)(*[f.ctypes.data for f in frags])
    if nthreads > 1:
        rc = lib().or_decode_mt(k, size, _ptr(rows), ptrs, _ptr(out), nthreads)
    else:
        rc = lib().or_decode(k, size, _ptr(rows), ptrs, _ptr(out))
    if rc != 0:
        raise ValueError("or_decode rejected")
    return out


def mask_rows(mask):
    """Brick mask -> ascending rows (brick_idx + 1), like ec-inode-read.c:1174."""
    return [i + 1 for i in range(64) if (mask >> i) & 1]


def writev_merge(k, head, user, old_head=None, old_tail=None):
    """The padded buffer a partial-stripe write encodes (test infrastructure).

    Restates ec_writev_prepare_buffers (ec-inode-write.c:1825-1848: a buffer
    of roundup(head + user, stripe) bytes with the user data at `head`),
    the zero fill beyond end of file (ec_writev_start, :2007-2008, :2031)
    and the old-stripe merges ec_merge_stripe_head_locked (:1883-1895: the
    head bytes and, for a one-stripe write, the bytes after the user data)
    and ec_merge_stripe_tail_locked (:1898-1908: the last `tail` bytes of the
    last stripe).  old_head / old_tail are stripe-sized arrays or None.
    """
    S = CHUNK * k
    user = np.asarray(user, dtype=np.uint8)
    us = user.size
    size = (head + us + S - 1) // S * S
    v = np.zeros(size, np.uint8)
    v[head:head + us] = user
    if size == S:
        old = old_head if old_head is not None else old_tail
        if old is not None:
            v[:head] = old[:head]
            v[head + us:] = old[head + us:S]
    else:
        if old_head is not None:
            v[:head] = old_head[:head]
        if old_tail is not None:
            tail = size - (head + us)
            v[head + us:] = old_tail[S - tail:S]
    return v
