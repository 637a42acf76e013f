"""Host timeline of the pipelined C3 forward: per chunk, when its ds_mat landed in pinned memory
and when its stage C (host Hungarian + selection/classifier launches) was queued, against the GPU
stage's end (HIP events) and the forward's end (synchronised).
    python tools/timeline.py [B] [n]"""
import os
import sys
import time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fpm  # noqa: E402
from fpm import params, synth  # noqa: E402
from fpm.batch import DeviceBatch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda", 0)
pairs = synth.make_batch(0, B, n)
bt = DeviceBatch.from_pairs(pairs, dev)
net = fpm.Net(regression=True, backbone=False, dtype="bf16")
net.load_state_dict(params.init_params(0))
for it in range(6):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    net.run(bt)
    torch.cuda.synchronize()
    tot = (time.perf_counter() - t0) * 1e3
    lt = net.last_timing
    if it >= 2:
        print("forward %.2f ms  gpu_stage %.2f ms  lsa %.2f ms  enqueue %.2f ms  chunks %d" % (
            tot, lt["gpu_stage_s"] * 1e3, lt["lsa_s"] * 1e3, lt["enqueue_s"] * 1e3, lt["chunks"]))
        print("   ready/queued:", " ".join("%.1f/%.1f" % x for x in lt["chunk_timeline_ms"]))
