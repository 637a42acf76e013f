"""Isolated timing of the AFA-U cross-set attention kernel (fpm_crossset_attn_fwd) at C3 chunk size:
python tools/attn_bench.py [B] [n]  -> ms per launch for the score LUT on / off."""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import fpm
from fpm import ops, params

DEV = torch.device("cuda", 0)
B, n = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (128, 256)
sd = params.init_params(7)
net = fpm.Net(regression=True, backbone=False, dtype="bf16")
net.load_state_dict(sd)
wp = net.packed(DEV)
g = torch.Generator().manual_seed(0)
ss = torch.softmax(torch.randn(B, n, n, generator=g) * 3, -1).to(DEV)
n2 = torch.full((B,), n, dtype=torch.int32, device=DEV)
out = torch.empty(B * n, 768, device=DEV, dtype=torch.bfloat16)
args = (ss, n2, wp["row_Wv"], wp["row_mix1w"], wp["row_mix1b"], wp["row_mix2w"], wp["row_mix2b"], out)
for lut in (1, 0, 1, 0):
    ops.set_tuning("afau_lut", lut)   # 0: the LDS-V kernel (interval-classified scores in bf16)
    for _ in range(3):
        ops.crossset_attn(*args, split=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.crossset_attn(*args, split=True)
    e1.record()
    torch.cuda.synchronize()
    print("lut", lut, "ms per launch %.4f" % (e0.elapsed_time(e1) / 20))
