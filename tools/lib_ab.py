"""Bit-identity and timing of one op between the in-tree library and another build of it
(e.g. the previous commit's, saved under tools/_ab/):  python tools/lib_ab.py <other.so> [afau]

Runs the AFA-U forward (Net._afau) on a seeded C3 chunk with each library in a child process and
compares the outputs bit for bit."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, os
sys.path.insert(0, %r)
import torch
import fpm
from fpm import _lib, params, synth
from fpm.batch import DeviceBatch
if sys.argv[1] != "-":
    _lib.LIB_PATH = sys.argv[1]
dev = torch.device("cuda", 0)
B, n = 128, 256
bt = DeviceBatch.from_pairs(synth.make_batch(5, B, n), dev)
net = fpm.Net(regression=True, backbone=False, dtype="bf16")
net.load_state_dict(params.init_params(0))
g = torch.Generator(device="cpu").manual_seed(3)
ss = torch.rand(B, n, n, generator=g) ** 6
ss = (ss / ss.sum(-1, keepdim=True)).to(dev)
wp = net.packed(dev)
ks = net._afau(wp, ss, bt)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    net._afau(wp, ss, bt)
e1.record()
torch.cuda.synchronize()
torch.save(ks.cpu(), sys.argv[2])
print("afau ms %%.3f" %% (e0.elapsed_time(e1) / 10))
""" % REPO

outs = []
for lib in ("-", sys.argv[1]):
    path = "/tmp/lib_ab_%d.pt" % len(outs)
    r = subprocess.run([sys.executable, "-c", CHILD, lib, path], capture_output=True, text=True, timeout=300)
    print(("in-tree " if lib == "-" else "other   ") + r.stdout.strip(), r.stderr[-400:] if r.returncode else "")
    if r.returncode:
        sys.exit(1)
    outs.append(path)
import torch  # noqa: E402
a, b = torch.load(outs[0]), torch.load(outs[1])
print("identical:", torch.equal(a, b), "max|diff| %.3g" % float((a - b).abs().max()))
