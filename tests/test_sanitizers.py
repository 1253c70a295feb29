"""SURVEY.md 5 (race detection / sanitizers; reference: configure --enable-asan
/ --enable-tsan, configure.ac:283-310): the host-only part of the library --
ec_method.c (GF(2^8), matrices, the LRU cache of inverses, the on-disk config
guard) and the CPU engine -- built with ASan+UBSan and with TSan around a
device-layer stub, then driven by 8 threads sharing one list with a 3-entry
cache (tests/c/sanitize_check.c).  CPU only; each build takes seconds."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "glusterfs_amd", "csrc")


def build(tmp_path, san, main="sanitize_check"):
    cc = shutil.which("gcc")
    if cc is None:
        pytest.skip("gcc not installed")
    objs = []
    common = ["-g", "-O1", "-fno-omit-frame-pointer", "-fPIC", "-std=gnu11", "-pthread",
              "-I" + os.path.join(ROOT, "include"), "-I" + CSRC] + san
    srcs = [(os.path.join(CSRC, "ec_method.c"), []), (os.path.join(CSRC, "ec_cpu.c"), []),
            (os.path.join(ROOT, "tests", "c", "ecd_stub.c"), [])]
    kerns = [("base", []), ("avx2", ["-mavx2"]), ("avx512", ["-mavx512f"])]
    for i, (src, extra) in enumerate(srcs):
        o = str(tmp_path / ("s%d.o" % i))
        subprocess.run([cc, *common, *extra, "-c", src, "-o", o], check=True)
        objs.append(o)
    procs = []                          # the three kernel builds run in parallel
    for sfx, flags in kerns:
        o = str(tmp_path / ("k_%s.o" % sfx))
        procs.append(subprocess.Popen([cc, *common, "-Wno-psabi",
                                       "-fno-tree-loop-distribute-patterns", "-DECC_SFX=" + sfx,
                                       *flags, "-c", os.path.join(CSRC, "ec_cpu_kern.c"),
                                       "-o", o]))
        objs.append(o)
    assert all(p.wait() == 0 for p in procs)
    exe = str(tmp_path / main)
    subprocess.run([cc, *common, os.path.join(ROOT, "tests", "c", main + ".c"), *objs,
                    "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("san", [["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
                                 ["-fsanitize=thread"]], ids=["asan-ubsan", "tsan"])
def test_host_layer_under_sanitizers(tmp_path, san):
    exe = build(tmp_path, san)
    env = dict(os.environ, EC_MI355X_QUIET="1", ASAN_OPTIONS="detect_leaks=1",
               TSAN_OPTIONS="halt_on_error=1")
    env.pop("EC_GPU_ALWAYS", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "failures=0" in r.stdout, (r.stdout + r.stderr)[-4000:]
    # again with the stub's pretend device, near-tie costs and a fixed GPU
    # share: every >= 1 MiB call is split onto the helper threads (r05), which
    # learn split shares concurrently
    env.update(ECD_STUB_GPU="1", EC_HYBRID_SHARE="450", EC_CPU_ENC_GBPS_K2="6",
               EC_CPU_DEC_GBPS_K="4", EC_XOVER_ADAPT="1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "failures=0" in r.stdout, (r.stdout + r.stderr)[-4000:]
    assert "split calls" in r.stdout, r.stdout[-2000:]


def test_fork_after_split_calls(tmp_path):
    """a child forked after the parent's split calls starts
    its own split helpers (pthread_atfork), instead of queueing its GPU share
    for the parent's helper threads, which it does not have, and waiting
    forever.  Stub device, every >= 1 MiB call split; tests/c/fork_check.c."""
    exe = build(tmp_path, ["-O1"], main="fork_check")
    env = dict(os.environ, EC_MI355X_QUIET="1", ECD_STUB_GPU="1", EC_HYBRID_SHARE="450",
               EC_CPU_ENC_GBPS_K2="6", EC_CPU_DEC_GBPS_K="4")
    env.pop("EC_GPU_ALWAYS", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and "parent ok, child exit 0" in r.stdout, r.stdout + r.stderr
