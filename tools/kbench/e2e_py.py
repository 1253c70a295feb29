import sys, time
sys.path.insert(0, "/root/repo"); sys.argv = ["bench.py"]
import torch, bench, glusterfs_amd as g
dev = torch.device("cuda", 0); torch.cuda.set_device(0)
c = bench.Ctx(g, torch, dev)
for k, n in ((4, 6), (8, 12), (16, 20)):
    print(k, n, bench.run_e2e(c, k, n, 512 << 20, 3))
