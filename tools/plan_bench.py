import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
from fpm import ops, synth
from fpm.batch import DeviceBatch
dev = torch.device("cuda", 0)
for n in (256, 512):
    bt = DeviceBatch.from_pairs(synth.make_batch(3, 128, n), dev)
    for it in range(3):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        p = ops.spline_plan(bt.src[0], bt.dst[0], bt.pseudo[0], 128 * n, n)
        e1.record(); torch.cuda.synchronize()
        print(n, bt.E[0], "plan ms %.3f" % e0.elapsed_time(e1))
    s = bt.src[0].cpu(); print("  src sorted:", bool((s[1:] >= s[:-1]).all()), "first", s[:12].tolist())
