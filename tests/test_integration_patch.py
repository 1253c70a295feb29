"""The reference-side binding as a patch:
integration/glusterfs-ec-mi355x.patch must apply cleanly (-p1) to the
reference's xlators/cluster/ec/src/{Makefile.am, ec-method.h, ec-types.h,
ec.c, ec-inode-write.c} and libglusterfs/src/{iobuf.c, glusterfs/iobuf.h, libglusterfs.sym},
drop every coding-layer source from ec.la, link libec_mi355x, leave
ec-method.h including the library header after ec-types.h, keep every
header ec.c includes in the distributed header list, and register the
client's iobuf arenas with the coder (pinned, device-mapped: zero copy)
after their mmap and unregister them before their munmap, and let a write
code only the fragments of the bricks it goes to.  Works on a
scratch copy; skipped where the reference tree is absent (the GPU box)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCH = os.path.join(ROOT, "integration", "glusterfs-ec-mi355x.patch")
REF = "/root/reference"
SUB = os.path.join("xlators", "cluster", "ec", "src")
LIBSRC = os.path.join("libglusterfs", "src")
FILES = tuple(os.path.join(SUB, f) for f in ("Makefile.am", "ec-method.h", "ec-types.h",
                                             "ec.c", "ec-inode-write.c")) + \
    tuple(os.path.join(LIBSRC, f) for f in ("iobuf.c", os.path.join("glusterfs", "iobuf.h"),
                                           "libglusterfs.sym"))


@pytest.fixture
def scratch(tmp_path):
    if not os.path.isdir(os.path.join(REF, SUB)):
        pytest.skip("reference tree not present")
    if shutil.which("patch") is None:
        pytest.skip("patch(1) not installed")
    d = tmp_path / "ref"
    for f in FILES:
        (d / f).parent.mkdir(parents=True, exist_ok=True)
        shutil.copy(os.path.join(REF, f), d / f)
    return d


def test_patch_applies_cleanly(scratch):
    for args in (["--dry-run"], []):
        r = subprocess.run(["patch", "-p1", "--forward", "--batch", *args, "-i", PATCH],
                           cwd=scratch, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "FAILED" not in r.stdout and "offset" not in r.stdout, r.stdout


def test_patched_build_files(scratch):
    subprocess.run(["patch", "-p1", "--batch", "-i", PATCH], cwd=scratch, check=True,
                   capture_output=True)
    mk = (scratch / SUB / "Makefile.am").read_text()
    for gone in ("ec-method.c", "ec-galois.c", "ec-code.c", "ec-code-c.c", "ec-gf8.c",
                 "ec-code-intel.c", "ec-code-x64.c", "ec-code-sse.c", "ec-code-avx.c"):
        assert gone not in mk, gone
    assert "-lec_mi355x" in mk and "$(EC_MI355X)/include" in mk
    for kept in ("ec.c", "ec-heal.c", "ec-inode-write.c", "ec-inode-read.c"):
        assert "ec_sources += %s" % kept in mk or "ec_sources := %s" % kept in mk
    hdr = (scratch / SUB / "ec-method.h").read_text()
    inc = [l.strip() for l in hdr.splitlines() if l.startswith("#include")]
    assert inc == ['#include "ec-types.h"', "#include <ec_method.h>"], inc
    assert not re.search(r"\bec_method_\w+\s*\(", hdr)   # prototypes come from the library
    assert '"avx", "hip"}' in (scratch / SUB / "ec.c").read_text()


def test_patched_ec_includes_are_distributed(scratch):
    """every local header the patched ec.c includes is either in
    ec_headers (so `make dist` ships it) or provided by the library."""
    subprocess.run(["patch", "-p1", "--batch", "-i", PATCH], cwd=scratch, check=True,
                   capture_output=True)
    mk = (scratch / SUB / "Makefile.am").read_text()
    listed = set(re.findall(r"ec_headers [+:]= (\S+)", mk))
    src = (scratch / SUB / "ec.c").read_text()
    local = re.findall(r'^#include "([^"]+)"', src, re.M)
    assert "ec-code.h" not in local and "ec-galois.h" not in local
    for h in local:
        assert h in listed, h
    # nothing from the dropped coding headers is used by ec.c
    for sym in ("ec_code_", "ec_gf_mul", "ec_gf_div", "EC_CODE_"):
        assert sym not in src, sym


def test_patched_iobuf_arena_hooks(scratch):
    """the client's iobuf arenas are registered with the
    coder after mmap and unregistered before munmap (iobuf.c:124, :157)."""
    subprocess.run(["patch", "-p1", "--batch", "-i", PATCH], cwd=scratch, check=True,
                   capture_output=True)
    io = (scratch / LIBSRC / "iobuf.c").read_text()
    m = io.index("mmap(NULL, iobuf_arena->arena_size")
    assert io.index("iobuf_arena_reg(iobuf_arena->mem_base", m) > m
    u = io.index("munmap(iobuf_arena->mem_base")
    assert io.rindex("iobuf_arena_unreg(iobuf_arena->mem_base", 0, u) < u
    assert "iobuf_set_arena_hooks(struct iobuf_pool *iobuf_pool" in io
    hdr = (scratch / LIBSRC / "glusterfs" / "iobuf.h").read_text()
    assert "typedef int (*iobuf_arena_hook_t)(void *base, size_t size);" in hdr
    assert "iobuf_set_arena_hooks\n" in (scratch / LIBSRC / "libglusterfs.sym").read_text()
    ec = (scratch / SUB / "ec.c").read_text()
    # registration is deferred to the library's thread: the arena hook runs
    # under iobuf_pool->mutex (VERDICT r03 missing #1)
    assert "ec_method_host_register_async(base, size)" in ec
    assert "ec_method_host_register(base" not in ec
    assert "ec_method_host_unregister(base)" in ec
    assert "ec->iobuf_hooks = ec_iobuf_hooks_get(this, &ec->matrix);" in ec
    assert "ec_iobuf_hooks_put(this);" in ec
    assert "gf_boolean_t iobuf_hooks;" in (scratch / SUB / "ec-types.h").read_text()


def _c_body(src, name):
    """Text of the C function `name` (definition at column 0 to its closing
    brace at column 0)."""
    i = src.index("\n%s(" % name) + 1
    return src[i:src.index("\n}\n", i) + 2]


def test_patched_iobuf_data_allocator_covers_every_size_class(scratch):
    """VERDICT r03 missing #1: ec_buffer_alloc (ec-helpers.c:134-165) ->
    iobuf_get_page_aligned -> iobuf_get2 (iobuf.c:513-569) serves a request
    from one of three places, and every one must reach the coder's pinned
    memory: <= 128 KiB GF_MALLOC (iobuf_get_from_small), > 1 MiB GF_CALLOC
    (iobuf_get_from_stdalloc) -- both now ask the data allocator first --
    and the arenas in between (registered by the arena hooks).  Frees of
    those buffers go back through the allocator's free hook."""
    subprocess.run(["patch", "-p1", "--batch", "-i", PATCH], cwd=scratch, check=True,
                   capture_output=True)
    io = (scratch / LIBSRC / "iobuf.c").read_text()
    # the size split of iobuf_get2 is the reference's, untouched
    get2 = _c_body(io, "iobuf_get2")
    assert "page_size <= USE_IOBUF_POOL_IF_SIZE_GREATER_THAN" in get2
    assert "iobuf_get_from_small(page_size)" in get2
    assert "iobuf_get_from_stdalloc(iobuf_pool, page_size)" in get2
    assert "__iobuf_get(iobuf_pool, rounded_size, index)" in get2
    # <= 128 KiB: the allocator first, GF_MALLOC when it declines
    small = _c_body(io, "iobuf_get_from_small")
    a, m = small.index("data_alloc(page_size)"), small.index("GF_MALLOC(page_size")
    assert a < m and "if (!iobuf->free_ptr)" in small[a:m]
    # > 1 MiB: the allocator first, GF_CALLOC when it declines
    std = _c_body(io, "iobuf_get_from_stdalloc")
    a, c = std.index("data_alloc((page_size + GF_IOBUF_ALIGN_SIZE) - 1)"), std.index("GF_CALLOC(\n")
    assert a < c
    # ... and its memory is zeroed, as GF_CALLOC's is (fuse,
    # protocol/client and other users of > 1 MiB iobufs get calloc'd memory)
    z = std.index("memset(iobuf->free_ptr, 0, (page_size + GF_IOBUF_ALIGN_SIZE) - 1);")
    assert a < z < c
    # every free of a non-arena iobuf asks the free hook before GF_FREE
    fr = _c_body(io, "__iobuf_free")
    assert fr.index("data_free(iobuf->free_ptr)") < fr.index("GF_FREE(iobuf->free_ptr)")
    assert "iobuf_set_data_allocator(struct iobuf_pool *iobuf_pool" in io
    # 128 KiB < size <= 1 MiB: arena pages, registered after the mmap
    assert "iobuf_arena_reg(iobuf_arena->mem_base" in _c_body(io, "__iobuf_arena_alloc")
    hdr = (scratch / LIBSRC / "glusterfs" / "iobuf.h").read_text()
    assert "typedef void *(*iobuf_data_alloc_t)(size_t size);" in hdr
    assert "typedef int (*iobuf_data_free_t)(void *ptr);" in hdr
    assert "iobuf_set_data_allocator\n" in (scratch / LIBSRC / "libglusterfs.sym").read_text()
    ec = (scratch / SUB / "ec.c").read_text()
    assert "ec_method_buffer_get(size)" in ec and "ec_method_buffer_put(ptr)" in ec
    get = _c_body(ec, "ec_iobuf_hooks_get")
    assert "iobuf_set_data_allocator(this->ctx->iobuf_pool, ec_iobuf_data_alloc," in get
    put = _c_body(ec, "ec_iobuf_hooks_put")
    # the free hook is kept when the last volume goes (buffers still out)
    assert "iobuf_set_data_allocator(this->ctx->iobuf_pool, NULL,\n" in put
    assert "ec_iobuf_data_free);" in put


def test_patched_writev_encodes_only_target_bricks(scratch):
    """ec_writev_encode (ec-inode-write.c:2125-2138) codes the fragments of the
    bricks the write can be wound to: fop->mask (ec_child_select only clears
    its bits) plus the healing bricks it adds back (the fop's and its
    parent's), limited to the volume's nodes -- so a heal write
    (ec-heal.c:327-329, heal->bad) computes only the bad bricks' fragments."""
    subprocess.run(["patch", "-p1", "--batch", "-i", PATCH], cwd=scratch, check=True,
                   capture_output=True)
    src = (scratch / SUB / "ec-inode-write.c").read_text()
    body = _c_body(src, "ec_writev_encode")
    assert "ec_method_encode(" not in body
    assert "targets = fop->mask | fop->healing;" in body
    assert "targets |= fop->parent->healing;" in body
    assert "targets & ec->node_mask" in body
    assert "ec_method_encode_rows(&ec->matrix, fop->vector[0].iov_len," in body
    # the dispatch that follows the encode is the one whose mask this bounds
    mgr = _c_body(src, "ec_manager_writev")
    e = mgr.index("ec_writev_encode(fop);")
    assert mgr.index("ec_dispatch_all(fop);", e) - e < 80
