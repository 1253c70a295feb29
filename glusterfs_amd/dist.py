"""Stripe-range sharding across processes (one process per MI355X).

Stripes are independent, so an N-GPU job is a contiguous
stripe-range partition with no data-path collective.  The only collectives
here are control plane: a barrier around timed regions, the max over ranks of
the elapsed time, and an all-ranks-ok flag.  Backend: "nccl" (RCCL) when the
ranks own GPUs, "gloo" otherwise (CPU tests).
"""
import os


def env_rank():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def local_device_index():
    """GPU of this rank: LOCAL_RANK, unless EC_BENCH_DEVICE pins every rank
    to one device (multi-rank rehearsal on a one-GPU box, with gloo)."""
    forced = os.environ.get("EC_BENCH_DEVICE")
    return int(forced) if forced is not None else env_rank()[2]


def stripe_range(rank, world, nstripes, align=1):
    """Contiguous [s0, s1) of rank `rank`; boundaries are multiples of
    `align` (pattern groups) except the final end."""
    units = (nstripes + align - 1) // align
    s0 = min(nstripes, units * rank // world * align)
    s1 = min(nstripes, units * (rank + 1) // world * align)
    return s0, s1


def parse_cpulist(text):
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11} (sysfs cpulist format)."""
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        else:
            cpus.add(int(part))
    return cpus


def bind_to_node(node, sysfs="/sys/devices/system/node"):
    """Restrict this process (the calling thread and every thread it starts
    afterwards: the library's copy pool, the CPU engine's callers) to the
    CPUs of NUMA node `node` that it may already use.  Returns the CPU set
    now in force; unchanged when the node is unknown or shares no CPU."""
    aff = set(os.sched_getaffinity(0))
    if node is None or node < 0:
        return aff
    try:
        with open(os.path.join(sysfs, "node%d" % node, "cpulist")) as f:
            mine = aff & parse_cpulist(f.read())
    except OSError:
        return aff
    if mine and mine != aff:
        os.sched_setaffinity(0, mine)
        return mine
    return aff


class Group:
    """torch.distributed wrapper that degrades to no-ops for world == 1."""

    def __init__(self, backend=None):
        self.rank, self.world, self.local = env_rank()
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            if backend is None:
                backend = os.environ.get("EC_BENCH_BACKEND") or (
                    "nccl" if torch.cuda.is_available() else "gloo")
            if not dist.is_initialized():
                dist.init_process_group(backend=backend)
            self.dist = dist
            self.backend = backend
        else:
            self.backend = None

    def _dev(self):
        import torch
        if self.backend == "nccl":
            return torch.device("cuda", local_device_index())
        return torch.device("cpu")

    def barrier(self):
        if self.dist:
            if self.backend == "nccl":
                self.dist.barrier(device_ids=[local_device_index()])
            else:
                self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return float(x)
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64, device=self._dev())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def all_ok(self, ok):
        if not self.dist:
            return bool(ok)
        import torch
        t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=self._dev())
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return bool(t.item())

    def gather(self, obj):
        """Every rank's `obj` (a small picklable value), in rank order."""
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist and self.dist.is_initialized():
            self.barrier()
            self.dist.destroy_process_group()
