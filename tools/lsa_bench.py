"""Host-LSA micro-benchmark on ds_mat-like inputs (soft top-k output of the oracle, n = $N, 256).

    python tools/lsa_bench.py [label]        (FPM_LSA_SCALAR=1 selects the scalar solver)
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fpm import ops, params, synth  # noqa: E402
import oracle as O  # noqa: E402

torch.set_num_threads(16)
N = int(os.environ.get("N", 256))
cache = "/tmp/lsa_bench_ds_%d.npy" % N
if os.path.exists(cache):
    ds = np.load(cache)
else:
    ds = O.forward(synth.make_batch(0, 4, N), params.init_params(0))["ds_mat"].numpy()
    np.save(cache, ds)
big = torch.from_numpy(np.tile(ds, (256, 1, 1)).copy())
n = torch.full((1024,), N, dtype=torch.int32)
label = sys.argv[1] if len(sys.argv) > 1 else "default"
for th in (1, 16):
    m = 64 if th == 1 else 1024
    ops.lsa_batch_host(big[:16], n[:16], n[:16], th)
    t = time.perf_counter()
    ops.lsa_batch_host(big[:m], n[:m], n[:m], th)
    dt = time.perf_counter() - t
    print("%s threads %d: %.3f ms per pair per thread, %.1f ms per 1024 pairs" % (label, th, dt * 1e3 / m * th,
                                                                               dt * 1e3 / m * 1024), flush=True)
