"""Development probe: does initialising the HIP runtime (the library's
device discovery) change the process's CPU affinity or its CPU-bound
throughput?  Prints the affinity before / after and a 1-thread and
16-thread CPU-engine rate before / after."""
import ctypes
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["EC_MI355X_QUIET"] = "1"


def rate(L, data, frags, threads, secs=1.0):
    k, n = 4, 6
    nst = data.size // (512 * k) // threads
    stop = time.perf_counter() + secs
    done = [0] * threads

    def w(i):
        d = data[i * nst * 512 * k:]
        f = [x[i * nst * 512:] for x in frags]
        while time.perf_counter() < stop:
            L.encode_batch(nst, d, f)
            done[i] += 1

    th = [threading.Thread(target=w, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    return sum(done) * nst * 512 * k / (time.perf_counter() - t0) / 1e9


def main():
    import glusterfs_amd as g
    data = np.random.default_rng(1).integers(0, 256, 16 << 20, dtype=np.uint8)
    frags = [np.empty(data.size // 4, np.uint8) for _ in range(6)]
    with g.ECMatrixList(4, 6, gen="avx") as L:        # CPU engine, no HIP yet
        a0 = sorted(os.sched_getaffinity(0))
        r1, r16 = rate(L, data, frags, 1), rate(L, data, frags, 16)
        print("before HIP init: affinity %d cpus (%s..%s); 1 thr %.1f GB/s, 16 thr %.1f GB/s" %
              (len(a0), a0[0], a0[-1], r1, r16), flush=True)
        print("devices", g.device_count(), flush=True)  # initialises HIP
        a1 = sorted(os.sched_getaffinity(0))
        r1, r16 = rate(L, data, frags, 1), rate(L, data, frags, 16)
        print("after HIP init:  affinity %d cpus (%s..%s); 1 thr %.1f GB/s, 16 thr %.1f GB/s" %
              (len(a1), a1[0], a1[-1], r1, r16), flush=True)
        print("threads in process:", len(os.listdir("/proc/self/task")))


if __name__ == "__main__":
    main()
