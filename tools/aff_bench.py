"""Time the batched vertex-affinity GEMM (Kp^T per pair, softplus - 0.5 epilogue) alone at C3's
chunk shape: B pairs x (n2 x n1 x 768), bf16 operands, for the kernel variants given as
key=value tuning switches (interleaved rounds, median)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import fpm  # noqa: E402,F401
from fpm import ops  # noqa: E402

B, n, D = int(os.environ.get("B", 128)), int(os.environ.get("N", 256)), 768
dev = torch.device("cuda", 0)
x2 = (torch.randn(B * n, D, device=dev) * 0.05).to(torch.bfloat16)
x1 = (torch.randn(B * n, D, device=dev) * 0.05).to(torch.bfloat16)
nn_ = torch.full((B,), n, device=dev, dtype=torch.int32)
out = torch.empty(B, n, n, device=dev)
variants = [tuple((k, int(v)) for k, v in (kv.split("=") for kv in a.split(","))) for a in sys.argv[1:]] or [()]
res = {}
for rnd in range(5):
    for var in variants:
        prev = [(k, ops.set_tuning(k, v)) for k, v in var]
        run = lambda: ops.gemm(x2, x1, n, n, D, D, D, batch=B, sA=n * D, sB=n * D, epi=ops.EPI_AFFINITY, out_f=out,
                               ldc=n, sC=n * n, n1=nn_, n2=nn_)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(var, []).append(e0.elapsed_time(e1) / 20)
        if var == variants[0] and rnd == 0:
            ref = out.clone()
        elif rnd == 0:
            print(var, "max |d| vs first variant", float((out - ref).abs().max()))
        for k, v in prev:
            ops.set_tuning(k, v)
flop = 2.0 * B * n * n * D
for var, ts in res.items():
    ms = sorted(ts)[len(ts) // 2]
    print("%-30s median %.4f ms  %.0f TFLOP/s (%.3f of 2.5 PF)" % (var, ms, flop / (ms / 1e3) / 1e12,
                                                                flop / (ms / 1e3) / 2.5e15))
