"""ec_method_last_error() is per calling thread, and every failing entry
point leaves its thread a reason (CPU suite: the host layer's own failures;
the device layer's are in tests/test_gpu_errors.py).

The reference logs a coder failure on the thread that saw it (ec-method.c
callers in ec-common.c / ec-heal.c run on several epoll threads and the heal
syncenv); r04's process-wide slot handed one thread's text to another's log
line ("What's weak" 1-2)."""
import ctypes
import threading

import numpy as np
import pytest

CHUNK = 512


@pytest.fixture(scope="module")
def g():
    import glusterfs_amd as g
    return g


def last_error(g):
    return (g.ec_method.lib.ec_method_last_error() or b"").decode()


def test_failure_names_entry_point_and_errno(g):
    with g.ECMatrixList(4, 6) as L:
        frags = [np.zeros(CHUNK, np.uint8) for _ in range(4)]
        out = np.zeros(CHUNK * 4, np.uint8)
        with pytest.raises(OSError) as ei:
            L.decode_batch(1, 0b11, [1, 2], frags, out)      # 2 bits set, k = 4
        assert "ec_method_decode_batch" in str(ei.value)
        assert "Invalid argument" in last_error(g)
        assert "ec_method_decode_batch" in last_error(g)


def test_success_keeps_last_failure(g):
    """The text is the thread's last failure, not cleared by a success
    (a log line written after a fallback still says what failed)."""
    with g.ECMatrixList(4, 6) as L:
        with pytest.raises(OSError):
            L.heal(1, 0b1111, [np.zeros(CHUNK, np.uint8)] * 4, 0, [])   # no target
        before = last_error(g)
        assert "ec_method_heal" in before
        data = np.arange(CHUNK * 4, dtype=np.uint32).astype(np.uint8)
        L.encode_batch(1, data, [np.zeros(CHUNK, np.uint8) for _ in range(6)])
        assert last_error(g) == before


def test_last_error_is_per_thread(g):
    """Two threads fail in different entry points, then (after both have
    failed) each reads its own reason."""
    lib = g.ec_method.lib
    got, errs = {}, []
    bar = threading.Barrier(2)

    def a(L):
        try:
            frags = [np.zeros(CHUNK, np.uint8) for _ in range(4)]
            with pytest.raises(OSError):
                L.decode_batch(1, 0b11, [1, 2], frags, np.zeros(CHUNK * 4, np.uint8))
            bar.wait()
            bar.wait()
            got["a"] = (lib.ec_method_last_error() or b"").decode()
        except Exception as e:   # noqa: BLE001 -- reported below
            errs.append(e)

    def b(L):
        try:
            bar.wait()
            rc = lib.ec_method_decode_mixed(ctypes.byref(L._list), 8, 3, None, None, None)
            assert rc < 0                                        # group of 3 stripes
            bar.wait()
            got["b"] = (lib.ec_method_last_error() or b"").decode()
        except Exception as e:   # noqa: BLE001
            errs.append(e)

    with g.ECMatrixList(4, 6) as L:
        th = [threading.Thread(target=a, args=(L,)), threading.Thread(target=b, args=(L,))]
        for t in th:
            t.start()
        for t in th:
            t.join()
    assert not errs, errs
    assert "ec_method_decode_batch" in got["a"] and "decode_mixed" not in got["a"], got
    assert "ec_method_decode_mixed" in got["b"] and "decode_batch" not in got["b"], got


def test_thread_without_failure_reads_no_other_threads_text(g):
    lib = g.ec_method.lib
    with g.ECMatrixList(4, 6) as L:
        with pytest.raises(OSError):
            L.decode_batch(1, 0b11, [1, 2], [np.zeros(CHUNK, np.uint8)] * 4,
                           np.zeros(CHUNK * 4, np.uint8))
    seen = []
    t = threading.Thread(target=lambda: seen.append((lib.ec_method_last_error() or b"").decode()))
    t.start()
    t.join()
    assert "decode_batch" not in seen[0]
    if g.device_count() > 0:
        assert seen[0] == ""
