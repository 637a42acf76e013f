"""The fp64 k chain (csrc/precise.hip, Net.k_f64_nmax): everything after the vertex affinity Kp --
the three PYGNNLayers with their Sinkhorns (gnn.py:207-226), the readout (ngm.py:368-369), the final
Sinkhorn (ngm.py:371) and the AFA-U regressor (ngm.py:386-412, afau.py:54-300) -- in float64.

Oracle: oracle/ngm_oracle.py evaluated in float64 (the restatement; its fp32 evaluation is the
reference's own arithmetic).  The device keeps SplineConv and Kp in fp32, whose rounding moves k by
< 5e-6 even on the ill-conditioned image-derived pairs (tools/kprob_arith.py), so:
  * per-kernel tests: within 1e-12 (relative to the values' scale) of the fp64 oracle on the same
    fp64 inputs;
  * end to end: ss within 1e-6 and k_prob within 2e-5 of the fp64 oracle forward, on synthetic C1 /
    ragged batches; ds_mat / k_prob within the north-star 1e-4 of the fp32 oracle.
"""
import types

import numpy as np
import pytest
import torch

import fpm
from fpm import ops, params, synth
from fpm.batch import DeviceBatch
import oracle as O
from oracle import ngm_oracle as NO

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _i32(x):
    return torch.as_tensor(np.asarray(x), dtype=torch.int32, device=DEV)


@pytest.fixture(scope="module")
def sd():
    return params.init_params(7)


@pytest.mark.parametrize("n1s,n2s,iters", [
    ((8, 8, 8), (8, 8, 8), 10),
    ((32, 20, 32), (32, 32, 17), 20),            # dummy rows + a transposed pair
    ((64, 41, 64), (50, 64, 64), 10),
    ((128, 100), (97, 128), 20),
])
def test_sinkhorn_f64_vs_oracle(n1s, n2s, iters):
    """fp64 log Sinkhorn (pygm semantics) vs the oracle in float64: contiguous and strided views,
    fp32 and fp64 inputs, the fp32 copy."""
    g = torch.Generator().manual_seed(7 + iters + n1s[0])
    B, n1max, n2max = len(n1s), max(n1s), max(n2s)
    s = torch.randn(B, n1max, n2max, generator=g, dtype=torch.float64) * 0.3
    ref = O.pygm_sinkhorn(s, n1s, n2s, dummy_row=True, max_iter=iters, tau=0.01)
    o32 = torch.empty(B, n1max, n2max, device=DEV)
    out = torch.empty(B, n1max, n2max, device=DEV, dtype=torch.float64)
    ops.sinkhorn_f64(s.to(DEV), _i32(n1s), _i32(n2s), iters, 0.01, True, out=out, out32=o32)
    assert float((out.cpu() - ref).abs().max()) < 1e-12
    assert torch.equal(o32.cpu(), out.cpu().float())
    sT = s.transpose(1, 2).contiguous().to(DEV).transpose(1, 2)
    oT = torch.zeros(B, n2max, n1max, device=DEV, dtype=torch.float64).transpose(1, 2)
    ops.sinkhorn_f64(sT, _i32(n1s), _i32(n2s), iters, 0.01, True, out=oT)
    assert torch.equal(oT.cpu(), out.cpu())
    # fp32 input: the same as the fp64 run on the widened values
    s32 = s.float()
    ref32in = O.pygm_sinkhorn(s32.double(), n1s, n2s, dummy_row=True, max_iter=iters, tau=0.01)
    out32in = ops.sinkhorn_f64(s32.to(DEV), _i32(n1s), _i32(n2s), iters, 0.01, True)
    assert float((out32in.cpu() - ref32in).abs().max()) < 1e-12


def test_gnn_layers_f64_vs_oracle(sd):
    """Three PYGNNLayers in fp64 from a fp32 Kp (ragged pairs: padded-space diagonal, dummy rows,
    transposed Sinkhorns) against ngm_oracle.gnn_layer in float64 on the same Kp."""
    pairs = synth.make_batch(23, 3, [30, 24, 28], n2=[26, 30, 28])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    net = fpm.Net(regression=True, backbone=False)
    net.load_state_dict(sd)
    wp = net.packed(DEV)
    B, n1max, n2max = bt.B, bt.n1max, bt.n2max
    pl = net.plans(bt)
    csr1 = ops.plan_csr(pl[0], bt.E[0], B * n1max)
    csr2 = ops.plan_csr(pl[1], bt.E[1], B * n2max)
    g = torch.Generator().manual_seed(5)
    Kp = torch.zeros(B, 1, n2max, n1max)
    for b in range(B):
        Kp[b, 0, :bt.n_host[1][b], :bt.n_host[0][b]] = torch.rand(int(bt.n_host[1][b]), int(bt.n_host[0][b]), generator=g)
    X, Cin = Kp.to(DEV), 1
    zbuf = torch.empty(B, n2max, n1max, device=DEV, dtype=torch.float64)
    outs = []
    for l in range(3):
        Xn = torch.empty(B, 17, n2max, n1max, device=DEV, dtype=torch.float64)
        ops.gnn_layer_f64(X, Cin, B, n1max, n2max, csr1, csr2, bt.n1, bt.n2, wp["gnn%d" % l], Xn, zbuf)
        ops.sinkhorn_f64(zbuf.transpose(1, 2), bt.n1, bt.n2, 20, 0.01, True, out=Xn[:, 16].transpose(1, 2))
        outs.append(Xn.cpu())
        X, Cin = Xn, 17
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    for b in range(B):
        n1b, n2b = int(bt.n_host[0][b]), int(bt.n_host[1][b])
        ei1, ei2 = torch.as_tensor(pairs[b][0]["edge_index"]), torch.as_tensor(pairs[b][1]["edge_index"])
        agg = lambda x: NO.pattern_mean_factorized(x, ei1, ei2, n1max, n2max, n1b, n2b)
        x = Kp[b].double().reshape(1, -1).t()                          # (N, 1), p = j * n1max + i
        for l in range(3):
            x = NO.gnn_layer(x, sd64, l, agg, n1max, n2max, n1b, n2b)
            got = outs[l][b].reshape(17, -1).t()
            err = float((got - x).abs().max() / x.abs().max())
            assert err < 1e-12, (b, l, err)


def _tailview(n1, n2):
    n_host = [torch.tensor(n1, dtype=torch.int32), torch.tensor(n2, dtype=torch.int32)]
    return types.SimpleNamespace(B=len(n1), device=DEV, nmax=[max(n1), max(n2)], n=[t.to(DEV) for t in n_host],
                                 n_host=n_host, n1=n_host[0].to(DEV), n2=n_host[1].to(DEV), n1max=max(n1),
                                 n2max=max(n2))


@pytest.mark.parametrize("n1,n2", [([32, 32, 32], [32, 32, 32]), ([30, 24, 28], [26, 30, 28]), ([64, 17], [40, 64])])
def test_afau_f64_vs_oracle(sd, n1, n2):
    """AFA-U regressor in fp64 (row block attention / combine / norms / FFN, col block per distinct n2,
    heads) against ngm_oracle.afau_ks in float64 on the same fp64 ss (doubly-stochastic-like
    Sinkhorn outputs, zero outside each pair's block)."""
    B, n1max, n2max = len(n1), max(n1), max(n2)
    g = torch.Generator().manual_seed(sum(n1))
    s = torch.randn(B, n1max, n2max, generator=g, dtype=torch.float64) * 0.02
    ss = O.pygm_sinkhorn(s, n1, n2, dummy_row=True, max_iter=10, tau=0.01)
    sd64 = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    ref = O.afau_ks(ss, torch.tensor(n1), torch.tensor(n2), sd64)
    net = fpm.Net(regression=True, backbone=False)
    net.load_state_dict(sd)
    ks = net._afau_f64(net.packed(DEV), ss.to(DEV), _tailview(n1, n2))
    assert float((ks.cpu().double() - ref).abs().max()) < 1e-7      # fp32 output of an fp64 evaluation


def _forward(pairs, sd, dtype="f32", k_f64=64):
    net = fpm.Net(regression=True, backbone=False, dtype=dtype)
    net.load_state_dict(sd)
    net.k_f64_nmax = k_f64
    bt = DeviceBatch.from_pairs(pairs, DEV)
    calls = []
    orig = ops.gnn_layer_f64

    def spy(*a, **kw):
        calls.append(1)
        return orig(*a, **kw)
    ops.gnn_layer_f64 = spy
    try:
        res = net.run(bt)
    finally:
        ops.gnn_layer_f64 = orig
    assert bool(calls) == (k_f64 >= max(bt.nmax)), "the fp64 k chain ran iff the box is within k_f64_nmax"
    return res


@pytest.mark.parametrize("case", ["c1", "ragged", "n64"])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_forward_k_f64_vs_oracle64(sd, case, dtype):
    """End to end through Net.run with the fp64 k chain: ss / k_prob against the float64 oracle forward
    (the fp32 SplineConv + Kp are the only fp32 stages left: ss within 1e-6, k within 2e-5) and the
    north-star gate against the fp32 oracle.  bf16 mode: these boxes take the fp32 SplineConv products
    (sc_f32_nmax) -- the same inputs to the fp64 chain, so the same outputs bit for bit."""
    pairs = {"c1": lambda: synth.make_batch(1, 1, 32),
             "ragged": lambda: synth.make_batch(3, 3, [30, 24, 28], n2=[26, 30, 28]),
             "n64": lambda: synth.make_batch(2, 4, 64)}[case]()
    res = _forward(pairs, sd, dtype)
    r64 = O.forward(pairs, sd, dtype=torch.float64)
    r32 = O.forward(pairs, sd)
    assert float((res["ss"].cpu().double() - r64["ss"]).abs().max()) < 1e-6
    assert float((res["k_prob"].cpu().double() - r64["k_prob"]).abs().max()) < 2e-5
    for k in ("ss", "ds_mat", "k_prob"):
        assert float((res[k].cpu() - r32[k]).abs().max()) < 1e-4, k
    if dtype == "bf16":
        ref = _forward(pairs, sd, "f32")
        for k in ("s", "ss", "ds_mat", "k_prob", "perm_mat"):
            assert torch.equal(res[k], ref[k]), k


def test_k_f64_off_above_threshold(sd):
    """k_f64_nmax below the box: the fp32 chain runs (and gives the fp32-gated result)."""
    pairs = synth.make_batch(1, 2, 32)
    res = _forward(pairs, sd, "f32", k_f64=16)
    r32 = O.forward(pairs, sd)
    for k in ("ss", "ds_mat", "k_prob"):
        assert float((res[k].cpu() - r32[k]).abs().max()) < 1e-4, k


@pytest.mark.parametrize("k_f64", [64, 0])
def test_forward_tiny_and_lopsided_pairs(sd, k_f64):
    """Edge sizes the reference handles (build_graphs.py:77-100: fewer than 3 points -> fully
    connected): a 1-keypoint graph (no edges: every SplineConv max over an empty in-edge set is 0,
    torch_scatter's rule), 2- and 3-keypoint graphs, and lopsided pairs (1 x 5, 3 x 40, 40 x 3:
    dummy rows, transposed Sinkhorns, k = round(ks * 1)).  Both k chains (fp64 on the 40-keypoint
    box, and the fp32 chain with k_f64_nmax = 0) against the oracle: ss / k_prob / cls_prob within
    1e-4 of the fp32 oracle, perm_mat identical or a proven tie class.  ds_mat is gated like the
    image path's k (anchored at the fp64 oracle): on the 2- and 7-keypoint pairs the fp32 oracle's
    own ds_mat sits 2.3e-4 / 1.1e-4 from its fp64 value (its ss 1.2e-5 from it: the tau = 0.01 soft
    top-k amplifies), so per pair |ds_dev - ds_64| <= |ds_32 - ds_64| + 1e-4."""
    pairs = synth.make_batch(5, 5, [1, 2, 3, 40, 7], n2=[5, 2, 40, 3, 7])
    assert pairs[0][0]["edge_index"].shape[1] == 0 and pairs[1][0]["edge_index"].shape[1] == 2
    res = _forward(pairs, sd, "f32", k_f64=k_f64)
    ref = O.forward(pairs, sd)
    r64 = O.forward(pairs, sd, dtype=torch.float64)
    for k in ("ss", "k_prob", "cls_prob"):
        assert float((res[k].cpu() - ref[k]).abs().max()) < 1e-4, k
    for b in range(len(pairs)):
        d_dev = float((res["ds_mat"][b].cpu().double() - r64["ds_mat"][b]).abs().max())
        d_ref = float((ref["ds_mat"][b].double() - r64["ds_mat"][b]).abs().max())
        print("pair %d ds_mat: device %.2e, fp32 oracle %.2e from fp64" % (b, d_dev, d_ref))
        assert d_dev <= d_ref + 1e-4, (b, d_dev, d_ref)
    rep = O.compare.perm_report(res, ref, [p[0]["n"] for p in pairs], [p[1]["n"] for p in pairs])
    assert rep["counts"]["mismatch"] == 0, rep
    if k_f64:
        assert float((res["k_prob"].cpu().double() - r64["k_prob"]).abs().max()) < 2e-5


@pytest.mark.parametrize("n1s,n2s,kfrac", [
    ((8, 8, 8), (8, 8, 8), (0.5, 0.2, 0.9)),
    ((32, 20, 32), (32, 32, 17), (0.55, 0.7, 0.35)),
    ((64, 41), (50, 64), (0.61, 0.48)),
])
def test_soft_topk_f64_vs_oracle(n1s, n2s, kfrac):
    """soft top-k in fp64 (csrc/precise.hip; the 2-column Sinkhorn_m incl. its while loop) against
    ngm_oracle.soft_topk in float64 on the same fp64 ss: within 1e-6 (the fp32 cast of an fp64
    evaluation); the padding zero; the pinned host copy identical."""
    g = torch.Generator().manual_seed(sum(n1s) + 3)
    B, n1max, n2max = len(n1s), max(n1s), max(n2s)
    s = torch.randn(B, n1max, n2max, generator=g, dtype=torch.float64) * 0.02
    ss = O.pygm_sinkhorn(s, n1s, n2s, dummy_row=True, max_iter=10, tau=0.01)
    k = torch.tensor([f * min(a, b) for f, a, b in zip(kfrac, n1s, n2s)], dtype=torch.float32)
    ref = O.soft_topk(ss, k.double(), list(n1s), list(n2s))
    steps = torch.zeros(B, dtype=torch.int32, device=DEV)
    host = torch.zeros(B, n1max, n2max).pin_memory()
    out = ops.soft_topk_f64(ss.to(DEV), _i32(n1s), _i32(n2s), k.to(DEV), 10, 0.01, steps=steps, out_host=host)
    torch.cuda.synchronize()
    assert float((out.cpu().double() - ref).abs().max()) < 1e-6
    assert torch.equal(host, out.cpu())
    assert int(steps.min()) >= 10
