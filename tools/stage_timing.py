import os, sys, time
os.environ["FPM_STAGE_TIMING"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
t0 = time.perf_counter()
def log(*a): print("[%.1fs]" % (time.perf_counter() - t0), *a, flush=True)
B = int(sys.argv[1]); n = int(sys.argv[2]); dt = sys.argv[3]
import bench
pairs = bench.make_pairs(0, 0, B, n, 16)
log("gen done")
import torch, fpm
from fpm import params
from fpm.batch import DeviceBatch
dev = torch.device("cuda", 0)
net = fpm.Net(regression=True, backbone=False, dtype=dt)
net.load_state_dict(params.init_params(0))
bt = DeviceBatch.from_pairs(pairs, dev)
log("on device")
for it in range(3):
    net.stage_times = {}
    net.run(bt)
    log("iter", it, {k: round(v * 1e3, 2) for k, v in net.stage_times.items()})
