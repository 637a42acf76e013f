import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count(), flush=True)
import torch
print("torch threads default", torch.get_num_threads(), flush=True)
import bench
from fpm import params
import oracle as O
sd = params.init_params(0)
for th in (16,):
    torch.set_num_threads(th)
    pairs = bench.make_pairs(1, 0, 2, 256, 1)
    t = time.perf_counter(); O.forward(pairs[:1], sd); print("threads", th, "1 pair", time.perf_counter() - t, flush=True)
    t = time.perf_counter(); O.forward(pairs, sd); print("threads", th, "2 pairs", time.perf_counter() - t, flush=True)
