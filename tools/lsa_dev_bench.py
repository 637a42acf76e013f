"""Time the device LSA on the forward's own ds_mat (n=256): one launch over B pairs is bounded by
the slowest pair's latency; also the host pool on the same matrices."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import fpm
from fpm import ops, params, synth
from fpm.batch import DeviceBatch

dev = torch.device("cuda", 0)
n = int(os.environ.get("N", "256"))
B = int(os.environ.get("B", "256"))
net = fpm.Net(regression=True, backbone=False, dtype="bf16", lsa="host")
net.load_state_dict(params.init_params(0))
bt = DeviceBatch.from_pairs(synth.make_batch(0, B, n), dev)
ds = net.run(bt)["ds_mat"].contiguous()
host = ops.lsa_batch_host(ds.cpu(), bt.n_host[0], bt.n_host[1], nthreads=16)
for nb in (1, 16, 64, B):
    sub = ds[:nb]
    a, st = ops.lsa_batch_device(sub, bt.n1[:nb], bt.n2[:nb])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        a, st = ops.lsa_batch_device(sub, bt.n1[:nb], bt.n2[:nb])
    e1.record()
    torch.cuda.synchronize()
    ok = torch.equal(a.cpu(), host[:nb])
    t0 = time.perf_counter()
    ops.lsa_batch_host(ds[:nb].cpu(), bt.n_host[0][:nb], bt.n_host[1][:nb], nthreads=16)
    th = time.perf_counter() - t0
    print("n=%d pairs=%4d device %.2f ms  host(16 thr) %.2f ms  identical=%s" % (n, nb, e0.elapsed_time(e1) / 3, th * 1e3, ok))
