"""Python mirror of the disperse coder's C ABI (include/ec_method.h).

This is a thin ctypes layer over glusterfs_amd/lib/libec_mi355x.so with the
same names, argument meaning and error behaviour as the reference's
ec-method.h:31-46 (ec_method_init / fini / update / encode / decode), plus the
batched, mixed-pattern, heal and device-resident entry points.  Negative
errno returns become ``OSError(errno)``; ``ec_method_encode`` mirrors the
reference's ``void`` signature.

Buffers can be numpy arrays, torch tensors (host or device), ctypes buffers or
plain integer addresses.  All coding happens in the native library (gfx950
kernels, or its C CPU engine for host buffers); there is no Python coding
path: if the library is missing, importing this module raises.
"""
import ctypes
import errno
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# EC_MI355X_LIB: another build of the same library (same-box A/B runs of two
# builds, tools/ab_lib.sh); the product path is lib/libec_mi355x.so
LIB_PATH = os.environ.get("EC_MI355X_LIB") or os.path.join(HERE, "lib", "libec_mi355x.so")

EC_GF_BITS = 8
EC_GF_MOD = 0x11D
EC_METHOD_MAX_FRAGMENTS = 16
EC_METHOD_WORD_SIZE = 64
EC_METHOD_CHUNK_SIZE = EC_METHOD_WORD_SIZE * EC_GF_BITS
EC_MAX_NODES = 31

# Every symbol include/ec_method.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "ec_method_init", "ec_method_fini", "ec_method_update", "ec_method_encode",
    "ec_method_decode", "ec_method_encode_batch", "ec_method_decode_batch",
    "ec_method_decode_mixed", "ec_method_heal", "ec_method_encode_device",
    "ec_method_decode_device", "ec_method_decode_mixed_device",
    "ec_method_heal_device", "ec_method_sync_device", "ec_method_device_count",
    "ec_method_last_error", "ec_method_host_alloc", "ec_method_host_free",
    "ec_method_host_register", "ec_method_host_unregister",
    "ec_method_encode_matrix", "ec_method_inverse_matrix", "ec_method_gf_mul",
    "ec_method_gf_div", "ec_method_config_fill", "ec_method_config_pack",
    "ec_method_config_unpack", "ec_method_config_check", "ec_method_writev_encode",
    "ec_method_writev_encode_device", "ec_method_engine", "ec_method_get_stats",
    "ec_method_inject_device_faults", "ec_method_device_numa_node", "ec_method_copy_threads",
    "ec_method_host_register_async", "ec_method_host_register_flush", "ec_method_buffer_get",
    "ec_method_buffer_put", "ec_method_pool_stats", "ec_method_jit_stats",
    "ec_method_jit_compile_check", "ec_method_jit_prepare", "ec_method_xover_route",
    "ec_method_xover_split",
    "ec_method_xover_plan",
    "ec_method_xover_observe_split",
    "ec_method_xover_observe_part",
    "ec_method_xover_observe", "ec_method_xover_reset", "ec_method_encode_rows",
    "ec_method_encode_rows_device",
)


class MatrixList(ctypes.Structure):
    """ec_matrix_list_t storage (120 bytes, layout of ec-types.h:549-562)."""
    _fields_ = [
        ("lru", ctypes.c_void_p * 2),
        ("lock", ctypes.c_byte * 40),
        ("columns", ctypes.c_uint32),
        ("rows", ctypes.c_uint32),
        ("max", ctypes.c_uint32),
        ("count", ctypes.c_uint32),
        ("stripe", ctypes.c_uint32),
        ("pool", ctypes.c_void_p),
        ("gf", ctypes.c_void_p),
        ("code", ctypes.c_void_p),
        ("encode", ctypes.c_void_p),
        ("objects", ctypes.c_void_p),
    ]


assert ctypes.sizeof(MatrixList) == 120


class _IOVec(ctypes.Structure):
    _fields_ = [("iov_base", ctypes.c_void_p), ("iov_len", ctypes.c_size_t)]


def _nbytes(buf):
    """Byte length of a numpy array / torch tensor / bytes-like buffer."""
    if hasattr(buf, "nbytes"):
        return int(buf.nbytes)
    if hasattr(buf, "numel"):
        return int(buf.numel() * buf.element_size())
    return len(buf)


class Stats(ctypes.Structure):
    """ec_method_stats_t: process-wide engine counters."""
    _fields_ = [("gpu_calls", ctypes.c_uint64), ("cpu_calls", ctypes.c_uint64),
                ("cpu_fallbacks", ctypes.c_uint64)]


class JitStats(ctypes.Structure):
    """ec_method_jit_stats_t: per-pattern kernels compiled at run time."""
    _fields_ = [(n, ctypes.c_uint64) for n in
                ("compiled", "failed", "launches", "compile_us", "lookups", "entries")]


class PoolStats(ctypes.Structure):
    """ec_method_pool_stats_t: pinned buffer pool and deferred registration."""
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "pool_bytes", "in_use_bytes", "gets", "misses", "slabs", "slab_register_us",
        "deferred_registers", "deferred_register_us", "deferred_register_failures",
        "unregisters", "unregister_us")]


class Config(ctypes.Structure):
    """ec_config_t (ec-types.h:145-152): the trusted.ec.config fields."""
    _fields_ = [
        ("version", ctypes.c_uint32),
        ("algorithm", ctypes.c_uint8),
        ("gf_word_size", ctypes.c_uint8),
        ("bricks", ctypes.c_uint8),
        ("redundancy", ctypes.c_uint8),
        ("chunk_size", ctypes.c_uint32),
    ]

    def astuple(self):
        return (self.version, self.algorithm, self.gf_word_size, self.bricks,
                self.redundancy, self.chunk_size)


def _load():
    # One HIP runtime per process: the torch wheel bundles its own
    # libamdhip64.so.7, and libc10_hip links it by a different name, so if
    # this library were loaded first the process would end up with two HIP
    # runtimes (torch then reports no GPU).  Importing torch first makes the
    # dynamic loader bind our libamdhip64.so.7 dependency to torch's copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libec_mi355x.so not built (%s); run `make -C glusterfs_amd` or "
            "__graft_entry__.build() -- there is no CPU fallback" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
    up = ctypes.c_size_t  # uintptr_t
    P = ctypes.POINTER(MatrixList)
    sig = {
        "ec_method_init": (i32, [vp, P, u32, u32, u32, ctypes.c_char_p]),
        "ec_method_fini": (None, [P]),
        "ec_method_update": (i32, [vp, P, ctypes.c_char_p]),
        "ec_method_encode": (None, [P, u64, vp, vp]),
        "ec_method_encode_rows": (None, [P, u64, vp, up, vp]),
        "ec_method_encode_rows_device": (i32, [P, ctypes.c_int, vp, u64, vp, up, vp]),
        "ec_method_decode": (i32, [P, u64, up, vp, vp, vp]),
        "ec_method_encode_batch": (i32, [P, u64, vp, vp]),
        "ec_method_decode_batch": (i32, [P, u64, up, vp, vp, vp]),
        "ec_method_decode_mixed": (i32, [P, u64, u64, vp, vp, vp]),
        "ec_method_heal": (i32, [P, u64, up, vp, up, vp]),
        "ec_method_encode_device": (i32, [P, ctypes.c_int, vp, u64, vp, vp]),
        "ec_method_decode_device": (i32, [P, ctypes.c_int, vp, u64, up, vp, vp]),
        "ec_method_decode_mixed_device": (i32, [P, ctypes.c_int, vp, u64, u64, vp, u32, vp,
                                                vp, vp]),
        "ec_method_heal_device": (i32, [P, ctypes.c_int, vp, u64, up, vp, up, vp]),
        "ec_method_sync_device": (i32, [ctypes.c_int, vp]),
        "ec_method_device_count": (i32, []),
        "ec_method_device_numa_node": (i32, [i32]),
        "ec_method_copy_threads": (i32, []),
        "ec_method_last_error": (ctypes.c_char_p, []),
        "ec_method_host_alloc": (vp, [ctypes.c_size_t]),
        "ec_method_host_free": (None, [vp]),
        "ec_method_host_register": (ctypes.c_int32, [vp, ctypes.c_size_t]),
        "ec_method_host_unregister": (ctypes.c_int32, [vp]),
        "ec_method_host_register_async": (i32, [vp, ctypes.c_size_t]),
        "ec_method_host_register_flush": (None, []),
        "ec_method_buffer_get": (vp, [ctypes.c_size_t]),
        "ec_method_buffer_put": (i32, [vp]),
        "ec_method_pool_stats": (None, [ctypes.POINTER(PoolStats)]),
        "ec_method_jit_stats": (None, [ctypes.POINTER(JitStats)]),
        "ec_method_jit_compile_check": (i32, [u32, u32, vp, ctypes.POINTER(u32)]),
        "ec_method_jit_prepare": (i32, [u32, u32, vp]),
        "ec_method_xover_route": (i32, [u32, i32, u64, u64, u64, u64]),
        "ec_method_xover_split": (i32, [u32, i32, u64, u64, u64, u64]),
        "ec_method_xover_plan": (i32, [u32, i32, u64, u64, u64, u64, u32, ctypes.POINTER(i32)]),
        "ec_method_xover_observe_split": (i32, [i32, u32, u64, u64, u64, u32, u64, u64]),
        "ec_method_xover_observe_part": (i32, [i32, i32, u32, u64, u64, u64, u64, u64]),
        "ec_method_xover_observe": (i32, [i32, i32, u32, u64, u64]),
        "ec_method_xover_reset": (None, []),
        "ec_method_encode_matrix": (i32, [u32, u32, vp]),
        "ec_method_inverse_matrix": (i32, [u32, vp, vp]),
        "ec_method_gf_mul": (u32, [u32, u32]),
        "ec_method_gf_div": (u32, [u32, u32]),
        "ec_method_writev_encode": (i32, [P, u64, vp, ctypes.c_int, vp, vp, vp]),
        "ec_method_writev_encode_device": (i32, [P, ctypes.c_int, vp, u64, u64, vp, vp, vp,
                                                 vp]),
        "ec_method_config_fill": (None, [u32, u32, ctypes.POINTER(Config)]),
        "ec_method_config_pack": (i32, [ctypes.POINTER(Config), vp]),
        "ec_method_config_unpack": (i32, [vp, ctypes.c_size_t, ctypes.POINTER(Config)]),
        "ec_method_config_check": (i32, [u32, u32, ctypes.POINTER(Config)]),
        "ec_method_engine": (ctypes.c_char_p, [P]),
        "ec_method_get_stats": (None, [ctypes.POINTER(Stats)]),
        "ec_method_inject_device_faults": (None, [u32]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("EC_MI355X_LIB") and not hasattr(L, name):
            continue      # an older build under A/B (tools/ab_lib.sh): probes it lacks
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()


def addr(buf):
    """Address of a buffer: numpy array, torch tensor, ctypes object or int."""
    if buf is None:
        return None
    if isinstance(buf, int):
        return buf
    if hasattr(buf, "data_ptr"):          # torch.Tensor
        return buf.data_ptr()
    if hasattr(buf, "ctypes"):            # numpy.ndarray
        return buf.ctypes.data
    return ctypes.addressof(buf)


def _ptr_array(bufs):
    return (ctypes.c_void_p * len(bufs))(*[addr(b) for b in bufs])


def _check(rc, what):
    if rc != 0:
        err = -rc if rc < 0 else errno.EIO
        raise OSError(err, "%s failed: %s (%s)" % (what, os.strerror(err),
                                                   (lib.ec_method_last_error() or b"").decode()))
    return rc


def device_count():
    return lib.ec_method_device_count()


def device_numa_node(device):
    """NUMA node of gfx950 device `device` (-1: unknown / one-node host)."""
    return lib.ec_method_device_numa_node(device)


def copy_threads():
    """Staging copy threads of this process (ec_method_copy_threads)."""
    return lib.ec_method_copy_threads()


def stats():
    """Process-wide engine counters as a dict (ec_method_get_stats)."""
    st = Stats()
    lib.ec_method_get_stats(ctypes.byref(st))
    return dict(gpu_calls=st.gpu_calls, cpu_calls=st.cpu_calls, cpu_fallbacks=st.cpu_fallbacks)


def jit_stats():
    """Counters of the run-time compiled whole-matrix kernels."""
    st = JitStats()
    lib.ec_method_jit_stats(ctypes.byref(st))
    return {n: getattr(st, n) for n, _ in JitStats._fields_}


def jit_compile_check(k, rows, coef):
    """Compile (without a device) the kernel of a rows x k coefficient matrix:
    (code bytes or -errno, XOR instructions per dword column)."""
    import numpy as np
    c = np.ascontiguousarray(np.asarray(coef, dtype=np.uint8).reshape(rows, k))
    ops = ctypes.c_uint32(0)
    rc = lib.ec_method_jit_compile_check(k, rows, c.ctypes.data, ctypes.byref(ops))
    return rc, ops.value


def jit_prepare(k, rows, coef):
    """Queue the kernel of a rows x k coefficient matrix for compilation."""
    import numpy as np
    c = np.ascontiguousarray(np.asarray(coef, dtype=np.uint8).reshape(rows, k))
    return lib.ec_method_jit_prepare(k, rows, c.ctypes.data)


def pool_stats():
    """Pinned buffer pool / deferred registration counters as a dict."""
    st = PoolStats()
    lib.ec_method_pool_stats(ctypes.byref(st))
    return {n: getattr(st, n) for n, _ in PoolStats._fields_}


def inject_device_faults(count):
    """Test hook: the next `count` host-buffer device submissions fail."""
    lib.ec_method_inject_device_faults(count)


class PinnedArray:
    """numpy uint8 view of pinned, device-mapped host memory
    (ec_method_host_alloc): host buffers here are coded in place over PCIe."""

    def __init__(self, nbytes):
        import numpy as np
        self.nbytes = int(nbytes)
        self.ptr = lib.ec_method_host_alloc(max(1, self.nbytes))
        if not self.ptr:
            raise MemoryError("ec_method_host_alloc(%d)" % self.nbytes)
        raw = (ctypes.c_uint8 * max(1, self.nbytes)).from_address(self.ptr)
        self.array = np.ctypeslib.as_array(raw)[:self.nbytes]

    def free(self):
        if self.ptr:
            self.array = None
            lib.ec_method_host_free(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self.array

    def __exit__(self, *exc):
        self.free()

    def __del__(self):
        self.free()


class PoolBuffer:
    """numpy uint8 view of a buffer of the library's pinned pool
    (ec_method_buffer_get): what the integration patch's iobuf data allocator
    hands GlusterFS for its non-arena iobufs.  Falls back to a plain numpy
    array (pageable) when the pool returns NULL, as iobuf.c would fall back to
    GF_MALLOC; `pooled` says which."""

    def __init__(self, nbytes):
        import numpy as np
        self.nbytes = int(nbytes)
        self.ptr = lib.ec_method_buffer_get(max(1, self.nbytes))
        self.pooled = bool(self.ptr)
        if self.ptr:
            raw = (ctypes.c_uint8 * max(1, self.nbytes)).from_address(self.ptr)
            self.array = np.ctypeslib.as_array(raw)[:self.nbytes]
        else:
            self.array = np.empty(self.nbytes, np.uint8)

    def free(self):
        if self.ptr:
            self.array = None
            if lib.ec_method_buffer_put(self.ptr) != 1:
                raise RuntimeError("ec_method_buffer_put: not a pool buffer")
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class host_registered:
    """Context manager pinning an existing host buffer (ec_method_host_register)."""

    def __init__(self, buf):
        self.buf = buf
        self.ptr = addr(buf)
        self.nbytes = buf.nbytes

    def __enter__(self):
        _check(lib.ec_method_host_register(self.ptr, self.nbytes), "ec_method_host_register")
        return self.buf

    def __exit__(self, *exc):
        _check(lib.ec_method_host_unregister(self.ptr), "ec_method_host_unregister")


def gf_mul(a, b):
    return lib.ec_method_gf_mul(a, b)


def gf_div(a, b):
    return lib.ec_method_gf_div(a, b)


def encode_matrix(columns, rows):
    m = (ctypes.c_uint32 * (columns * rows))()
    _check(lib.ec_method_encode_matrix(columns, rows, m), "ec_method_encode_matrix")
    return [[m[i * columns + j] for j in range(columns)] for i in range(rows)]


def inverse_matrix(rows):
    k = len(rows)
    r = (ctypes.c_uint32 * k)(*rows)
    m = (ctypes.c_uint32 * (k * k))()
    _check(lib.ec_method_inverse_matrix(k, r, m), "ec_method_inverse_matrix")
    return [[m[i * k + j] for j in range(k)] for i in range(k)]


def mask_rows(mask):
    """Brick mask -> ascending rows (brick index + 1), as ec-inode-read.c:1174."""
    return [i + 1 for i in range(64) if (mask >> i) & 1]


class ECMatrixList:
    """An initialised ec_matrix_list_t: the coder of one disperse volume.

    Mirrors ec-method.h: ``ECMatrixList(columns=k, rows=n, max=2n, gen)`` is
    ec_method_init (ec.c:837), ``fini()`` ec_method_fini, ``encode`` and
    ``decode`` the two hot-path calls (ec-inode-write.c:2136,
    ec-inode-read.c:1196)."""

    def __init__(self, columns, rows, max=None, gen="auto"):
        self.columns, self.rows = columns, rows
        self.max = 2 * rows if max is None else max
        self._list = MatrixList()
        self._live = False
        rc = lib.ec_method_init(None, ctypes.byref(self._list), columns, rows, self.max,
                                gen.encode() if gen is not None else None)
        _check(rc, "ec_method_init")
        self._live = True

    # --- reference surface -------------------------------------------------
    @property
    def engine(self):
        return (lib.ec_method_engine(ctypes.byref(self._list)) or b"").decode()

    @property
    def stripe(self):
        return self._list.stripe

    @property
    def count(self):
        return self._list.count

    def fini(self):
        if self._live:
            lib.ec_method_fini(ctypes.byref(self._list))
            self._live = False

    def __del__(self):
        try:
            self.fini()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.fini()

    def update(self, gen):
        return _check(lib.ec_method_update(None, ctypes.byref(self._list), gen.encode()),
                      "ec_method_update")

    def encode(self, size, inp, out):
        """ec_method_encode: `out` is a list of n fragment buffers."""
        ptrs = _ptr_array(out)
        lib.ec_method_encode(ctypes.byref(self._list), size, addr(inp), ptrs)

    def encode_rows(self, size, inp, row_mask, out):
        """ec_method_encode_rows: `out` is a list of n fragment buffers (None
        where the bit of row_mask is clear); only the bricks in row_mask are
        computed."""
        lib.ec_method_encode_rows(ctypes.byref(self._list), size, addr(inp), row_mask,
                                  _ptr_array(out))

    def decode(self, size, mask, rows, inp, out):
        """ec_method_decode: size = bytes per fragment; rows = brick idx + 1."""
        r = (ctypes.c_uint32 * len(rows))(*rows)
        return _check(lib.ec_method_decode(ctypes.byref(self._list), size, mask, r,
                                           _ptr_array(inp), addr(out)), "ec_method_decode")

    # --- batched / new -------------------------------------------------------
    def encode_batch(self, nstripes, inp, out):
        return _check(lib.ec_method_encode_batch(ctypes.byref(self._list), nstripes,
                                                 addr(inp), _ptr_array(out)),
                      "ec_method_encode_batch")

    def decode_batch(self, nstripes, mask, rows, inp, out):
        r = (ctypes.c_uint32 * len(rows))(*rows)
        return _check(lib.ec_method_decode_batch(ctypes.byref(self._list), nstripes, mask, r,
                                                 _ptr_array(inp), addr(out)),
                      "ec_method_decode_batch")

    def decode_mixed(self, nstripes, group_stripes, group_masks, frags, out):
        gm = (ctypes.c_size_t * len(group_masks))(*group_masks)
        return _check(lib.ec_method_decode_mixed(ctypes.byref(self._list), nstripes,
                                                 group_stripes, gm, _ptr_array(frags),
                                                 addr(out)), "ec_method_decode_mixed")

    def writev_encode(self, head, user, old_head, old_tail, out):
        """ec_method_writev_encode: `user` is one buffer or a list of buffers
        (the writev iovec list); old_head / old_tail may be None."""
        bufs = user if isinstance(user, (list, tuple)) else [user]
        iov = (_IOVec * len(bufs))(*[_IOVec(addr(b), _nbytes(b)) for b in bufs])
        return _check(lib.ec_method_writev_encode(ctypes.byref(self._list), head, iov,
                                                  len(bufs), addr(old_head), addr(old_tail),
                                                  _ptr_array(out)), "ec_method_writev_encode")

    def writev_encode_device(self, device, stream, head, size, user, old_head, old_tail, out):
        return _check(lib.ec_method_writev_encode_device(
            ctypes.byref(self._list), device, stream, head, size, addr(user), addr(old_head),
            addr(old_tail), _ptr_array(out)), "ec_method_writev_encode_device")

    def heal(self, nstripes, mask, inp, target_mask, out):
        return _check(lib.ec_method_heal(ctypes.byref(self._list), nstripes, mask,
                                         _ptr_array(inp), target_mask, _ptr_array(out)),
                      "ec_method_heal")

    # --- device-resident, asynchronous --------------------------------------
    def encode_rows_device(self, device, stream, nstripes, inp, row_mask, out):
        """ec_method_encode_rows_device: out[i] (None where the bit of
        row_mask is clear) on device `device`, queued on `stream`."""
        return _check(lib.ec_method_encode_rows_device(ctypes.byref(self._list), device, stream,
                                                       nstripes, addr(inp), row_mask,
                                                       _ptr_array(out)),
                      "ec_method_encode_rows_device")

    def encode_device(self, device, stream, nstripes, inp, out):
        return _check(lib.ec_method_encode_device(ctypes.byref(self._list), device, stream,
                                                  nstripes, addr(inp), _ptr_array(out)),
                      "ec_method_encode_device")

    def decode_device(self, device, stream, nstripes, mask, inp, out):
        return _check(lib.ec_method_decode_device(ctypes.byref(self._list), device, stream,
                                                  nstripes, mask, _ptr_array(inp),
                                                  addr(out)), "ec_method_decode_device")

    def decode_mixed_device(self, device, stream, nstripes, group_stripes, group_pattern,
                            masks, frags, out):
        m = (ctypes.c_size_t * len(masks))(*masks)
        return _check(lib.ec_method_decode_mixed_device(
            ctypes.byref(self._list), device, stream, nstripes, group_stripes,
            addr(group_pattern), len(masks), m, _ptr_array(frags), addr(out)),
            "ec_method_decode_mixed_device")

    def heal_device(self, device, stream, nstripes, mask, inp, target_mask, out):
        return _check(lib.ec_method_heal_device(ctypes.byref(self._list), device, stream,
                                                nstripes, mask, _ptr_array(inp), target_mask,
                                                _ptr_array(out)), "ec_method_heal_device")


def sync_device(device, stream=None):
    return _check(lib.ec_method_sync_device(device, stream), "ec_method_sync_device")


# --- on-disk format guard (trusted.ec.config) ------------------------------
def config_fill(bricks, redundancy):
    """The Config a write stores (ec-dir-write.c:144-151)."""
    c = Config()
    lib.ec_method_config_fill(bricks, redundancy, ctypes.byref(c))
    return c


def config_pack(config):
    """8-byte big-endian xattr value (ec_dict_set_config)."""
    out = (ctypes.c_uint8 * 8)()
    _check(lib.ec_method_config_pack(ctypes.byref(config), out), "ec_method_config_pack")
    return bytes(out)


def config_unpack(value):
    """Parse an xattr value (ec_dict_del_config); OSError(ENODATA) if all 0."""
    c = Config()
    buf = ctypes.create_string_buffer(bytes(value), len(value))
    _check(lib.ec_method_config_unpack(buf, len(value), ctypes.byref(c)),
           "ec_method_config_unpack")
    return c


def config_check(bricks, redundancy, config):
    """ec_config_check: 0, -EINVAL (corrupted) or -ENOTSUP (other layout)."""
    return lib.ec_method_config_check(bricks, redundancy, ctypes.byref(config))
