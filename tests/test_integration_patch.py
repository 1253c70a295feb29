"""The reference-side binding as a patch:
integration/glusterfs-ec-mi355x.patch must apply cleanly (-p1) to the
reference's xlators/cluster/ec/src/{Makefile.am, ec-method.h, ec.c}, drop
every coding-layer source from ec.la, link libec_mi355x, and leave
ec-method.h including the library header after ec-types.h.  Works on a
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
FILES = ("Makefile.am", "ec-method.h", "ec.c")


@pytest.fixture
def scratch(tmp_path):
    if not os.path.isdir(os.path.join(REF, SUB)):
        pytest.skip("reference tree not present")
    if shutil.which("patch") is None:
        pytest.skip("patch(1) not installed")
    d = tmp_path / "ref"
    (d / SUB).mkdir(parents=True)
    for f in FILES:
        shutil.copy(os.path.join(REF, SUB, f), d / SUB / f)
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
