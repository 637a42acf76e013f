"""Time the spline plan (global vs per-graph kernels) on a C3 chunk:
   python tools/plan_bench.py plan_graph=0 plan_graph=1 ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fpm  # noqa: E402,F401
from fpm import ops, synth  # noqa: E402
from fpm.batch import DeviceBatch  # noqa: E402

dev = torch.device("cuda", 0)
B, n = int(os.environ.get("B", 128)), int(os.environ.get("N", 256))
bt = DeviceBatch.from_pairs(synth.make_batch(3, B, n), dev)
me = bt.max_graph_edges(0)
variants = [tuple((k, int(v)) for k, v in (kv.split("=") for kv in a.split(","))) for a in sys.argv[1:]] or [()]
res = {}
for rnd in range(5):
    for var in variants:
        prev = [(k, ops.set_tuning(k, v)) for k, v in var]
        ops.spline_plan(bt.src[0], bt.dst[0], bt.pseudo[0], B * n, n, me)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            ops.spline_plan(bt.src[0], bt.dst[0], bt.pseudo[0], B * n, n, me)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(var, []).append(e0.elapsed_time(e1) / 10)
        for k, v in prev:
            ops.set_tuning(k, v)
for var, ts in res.items():
    print("%-40s median %.4f ms" % (var, sorted(ts)[len(ts) // 2]))
