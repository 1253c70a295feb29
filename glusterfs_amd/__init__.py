"""glusterfs_amd -- MI355X-native drop-in for GlusterFS's disperse (EC) coder.

The product is the C-ABI library lib/libec_mi355x.so (include/ec_method.h);
this package is its Python mirror (ctypes) used by tests and bench.py.
"""
from .ec_method import (  # noqa: F401
    EC_METHOD_CHUNK_SIZE,
    EC_METHOD_MAX_FRAGMENTS,
    ECMatrixList,
    PinnedArray,
    PoolBuffer,
    copy_threads,
    device_count,
    device_numa_node,
    encode_matrix,
    gf_div,
    gf_mul,
    host_registered,
    jit_compile_check,
    jit_prepare,
    jit_stats,
    inject_device_faults,
    inverse_matrix,
    mask_rows,
    pool_stats,
    stats,
    sync_device,
)
