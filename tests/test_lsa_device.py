"""Device Hungarian (fpm_lsa_batch_device) vs the host solver and scipy.

The device kernel restates the host solver's algorithm (same arithmetic, scan order and tie rule),
so the bar is identical assignments on every input, including tie-heavy and all-zero matrices,
ragged and transposed (n2 < n1) pairs, the reference's golden Hungarian case and the forward's own
ds_mat at n = 256 / 512; and identical forward outputs with lsa="device" vs lsa="host".
"""
import os

import numpy as np
import pytest
import scipy.optimize as opt
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _scipy(s, n1, n2):
    r, c = opt.linear_sum_assignment(s[:n1, :n2] * -1)
    a = -np.ones(s.shape[0], np.int32)
    a[r] = c
    return a


def _mats(mode, B, n1max, n2max, seed):
    rng = np.random.default_rng(seed)
    s = np.zeros((B, n1max, n2max), np.float32)
    n1 = rng.integers(1, n1max + 1, B).astype(np.int32)
    n2 = rng.integers(1, n2max + 1, B).astype(np.int32)
    n1[0], n2[0] = n1max, n2max
    for b in range(B):
        if mode == "rand":
            blk = rng.random((n1[b], n2[b]))
        elif mode == "ties":
            blk = rng.integers(0, 3, (n1[b], n2[b]))
        elif mode == "zeros":
            blk = np.zeros((n1[b], n2[b]))
        else:
            blk = rng.random((n1[b], n2[b])) ** 8
            blk[blk < 0.3] = 0
        s[b, :n1[b], :n2[b]] = blk
    return s, n1, n2


@pytest.mark.parametrize("mode", ["rand", "ties", "zeros", "sparse"])
@pytest.mark.parametrize("n1max,n2max", [(37, 41), (70, 20), (130, 129)])
def test_lsa_device_matches_host(mode, n1max, n2max):
    from fpm import ops
    s, n1, n2 = _mats(mode, 24, n1max, n2max, {"rand": 1, "ties": 2, "zeros": 3, "sparse": 4}[mode] * 1000 + n1max)
    host = ops.lsa_batch_host(torch.from_numpy(s), torch.from_numpy(n1), torch.from_numpy(n2), nthreads=4)
    a, st = ops.lsa_batch_device(torch.from_numpy(s).to(DEV), torch.from_numpy(n1).to(DEV),
                                 torch.from_numpy(n2).to(DEV))
    assert not st.cpu().any()
    assert torch.equal(a.cpu(), host)
    for b in range(0, 24, 5):
        np.testing.assert_array_equal(a[b].cpu().numpy(), _scipy(s[b], n1[b], n2[b]))


def test_lsa_device_golden():
    from fpm import ops
    z = np.load(os.path.join(GOLDEN, "hungarian_greedy.npz"))
    a, st = ops.lsa_batch_device(torch.from_numpy(z["s"]).to(DEV), torch.from_numpy(z["n1"]).int().to(DEV),
                                 torch.from_numpy(z["n2"]).int().to(DEV))
    x = np.zeros_like(z["x"])
    for b, row in enumerate(a.cpu().tolist()):
        for r, c in enumerate(row):
            if c >= 0:
                x[b, r, c] = 1
    np.testing.assert_array_equal(x, z["x"])


def test_lsa_device_invalid_and_empty():
    from fpm import ops
    s = np.random.default_rng(3).random((3, 8, 8)).astype(np.float32)
    s[1, 2, 3] = np.nan
    s[2, 0, 0] = np.inf        # cost -inf: scipy rejects
    n1 = torch.tensor([0, 8, 8], dtype=torch.int32, device=DEV)
    n2 = torch.tensor([8, 8, 8], dtype=torch.int32, device=DEV)
    a, st = ops.lsa_batch_device(torch.from_numpy(s).to(DEV), n1, n2)
    assert st.cpu().tolist() == [0, 2, 2]
    assert (a[0].cpu() == -1).all()


@pytest.mark.parametrize("n,B", [(256, 12), (512, 4)])
def test_lsa_device_on_forward_ds_mat(n, B):
    """The forward's own ds_mat (soft top-k output, near-ties everywhere): device == host."""
    import fpm
    from fpm import ops, params, synth
    from fpm.batch import DeviceBatch
    net = fpm.Net(regression=True, backbone=False, dtype="bf16", lsa="host")
    net.load_state_dict(params.init_params(2))
    bt = DeviceBatch.from_pairs(synth.make_batch(4, B, n), DEV)
    res = net.run(bt)
    ds = res["ds_mat"]
    host = ops.lsa_batch_host(ds.cpu(), bt.n_host[0], bt.n_host[1], nthreads=4)
    a, st = ops.lsa_batch_device(ds, bt.n1, bt.n2)
    assert not st.cpu().any()
    assert torch.equal(a.cpu(), host)


def test_forward_device_lsa_equals_host_lsa():
    import fpm
    from fpm import params, synth
    from fpm.batch import DeviceBatch
    sd = params.init_params(6)
    pairs = synth.make_batch(12, 9, 64, n2=[64, 50, 64, 64, 40, 64, 61, 64, 64])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    outs = []
    for mode in ("host", "device"):
        net = fpm.Net(regression=True, backbone=False, lsa=mode)
        net.load_state_dict(sd)
        outs.append(net.run(bt, chunks=3))
    for k in ("ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert torch.equal(outs[0][k], outs[1][k]), k
