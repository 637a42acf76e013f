"""Parity of the HIP path (through the C-ABI) against the CPU oracle on identical inputs.

Tolerances (fp32 mode): 1e-4 abs on ss / ds_mat / k_prob (the north-star gate), identical
perm_mat; per-stage tolerances are tighter where the stage is well conditioned.  The bf16 mode
is reported against the fp32 oracle with a loose bound (it is a throughput mode).
"""
import os

import numpy as np
import pytest
import torch

import fpm
from fpm import _lib, ops, params, synth
from fpm.batch import DeviceBatch
import oracle as O

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _i32(x):
    return torch.as_tensor(np.asarray(x), dtype=torch.int32, device=DEV)


@pytest.fixture(scope="module")
def sd():
    return params.init_params(7)


# ---------------------------------------------------------------------------------------- sinkhorn
@pytest.mark.parametrize("n1s,n2s,iters,tau", [
    ((8, 8, 8), (8, 8, 8), 10, 0.05),
    ((32, 20, 32), (32, 32, 17), 20, 0.01),          # dummy rows + transposed pair
    ((100, 64, 128), (128, 128, 90), 10, 0.01),
    ((256, 256), (256, 256), 20, 0.01),
    ((200, 256, 131), (256, 190, 256), 10, 0.01),
])
@pytest.mark.parametrize("lform", [1, 0])
def test_sinkhorn_vs_oracle(n1s, n2s, iters, tau, lform):
    """Register-tile forwards (lform 1: L-form, 0: potential form) against the float64 oracle."""
    g = torch.Generator().manual_seed(len(n1s) * 100 + n1s[0])
    B = len(n1s)
    n1max, n2max = max(n1s), max(n2s)
    s = torch.randn(B, n1max, n2max, generator=g) * 0.3
    ref = O.pygm_sinkhorn(s.double(), n1s, n2s, dummy_row=True, max_iter=iters, tau=tau)
    prev = ops.set_tuning("sinkhorn_lform", lform)
    try:
        out = ops.sinkhorn(s.to(DEV), _i32(n1s), _i32(n2s), iters, tau, True).cpu()
        # strided (transposed) input and output views
        sT = s.transpose(1, 2).contiguous().to(DEV).transpose(1, 2)
        o2 = torch.zeros(B, n2max, n1max, device=DEV).transpose(1, 2)
        ops.sinkhorn(sT, _i32(n1s), _i32(n2s), iters, tau, True, out=o2)
    finally:
        ops.set_tuning("sinkhorn_lform", prev)
    assert (out.double() - ref).abs().max() < 1e-4
    assert (o2.cpu().double() - ref).abs().max() < 1e-4


@pytest.mark.parametrize("lform", [1, 0])
@pytest.mark.parametrize("form", [0, 1])
@pytest.mark.parametrize("n1s,n2s,iters,tau,scale", [
    ((256, 200, 131), (256, 256, 240), 20, 0.001, 0.1),    # small tau: shifted sums out of range -> max-shifted
                                                            # (|S / tau| <= ~430 log2 units: fp32 conditioning ~3e-5)
    ((240, 256), (256, 97), 20, 0.05, -2.0),                # one column + one row far below the rest:
                                                            # their lines underflow against the shifts
    ((64, 50), (64, 64), 1, 0.05, 0.3),                     # a single (log-domain) step
    ((128, 128, 77), (128, 60, 128), 21, 0.02, 1.0),        # odd step count, dummy rows, transposed pair
])
def test_sinkhorn_forms_vs_oracle(form, n1s, n2s, iters, tau, scale, lform):
    """Both Sinkhorn step forms (0 max-shifted log, 1 shifted single-pass lse with its range guard)
    against the float64 oracle, incl. inputs that trip the guards
    (scale < 0: |scale| x randn with column 3 and row 5 set to -6, ~330 log2 units below the
    row maxima)."""
    g = torch.Generator().manual_seed(31 + iters + len(n1s))
    B, n1max, n2max = len(n1s), max(n1s), max(n2s)
    s = torch.randn(B, n1max, n2max, generator=g) * abs(scale)
    if scale < 0:
        s[:, :, 3] = -6.0
        s[:, 5, :] = -6.0
    ref = O.pygm_sinkhorn(s.double(), n1s, n2s, dummy_row=True, max_iter=iters, tau=tau)
    prev = ops.set_tuning("sinkhorn_fast", form)
    prev_l = ops.set_tuning("sinkhorn_lform", lform)
    try:
        out = ops.sinkhorn(s.to(DEV), _i32(n1s), _i32(n2s), iters, tau, True).cpu()
        sT = s.transpose(1, 2).contiguous().to(DEV).transpose(1, 2)
        o2 = torch.zeros(B, n2max, n1max, device=DEV).transpose(1, 2)
        ops.sinkhorn(sT, _i32(n1s), _i32(n2s), iters, tau, True, out=o2)
    finally:
        ops.set_tuning("sinkhorn_fast", prev)
        ops.set_tuning("sinkhorn_lform", prev_l)
    assert (out.double() - ref).abs().max() < 1e-4
    assert (o2.cpu().double() - ref).abs().max() < 1e-4


# ---------------------------------------------------------------------------------------- soft top-k
def test_soft_topk_golden():
    z = np.load(os.path.join(GOLDEN, "soft_topk.npz"))
    for i in range(int(z["ncases"])):
        g = lambda k: z["c%d_%s" % (i, k)]
        sc = torch.from_numpy(g("scores")).to(DEV)
        out = ops.soft_topk_fwd(sc, _i32(g("n1")), _i32(g("n2")), torch.from_numpy(g("ks")).to(DEV), 10, 0.01)
        np.testing.assert_allclose(out.cpu().numpy(), g("ss_out"), atol=1e-5, rtol=0)


def test_soft_topk_vs_oracle_large():
    g = torch.Generator().manual_seed(5)
    B, n = 4, 256
    ss = torch.rand(B, n, n, generator=g) ** 6
    k = torch.tensor([30.5, 100.0, 5.2, 250.0])
    nn_ = [n] * B
    ref = O.soft_topk(ss, k, nn_, nn_, 10, 0.01)
    out = ops.soft_topk_fwd(ss.to(DEV), _i32(nn_), _i32(nn_), k.to(DEV), 10, 0.01).cpu()
    assert (out - ref).abs().max() < 1e-4


def test_soft_topk_stream_dense_and_ragged_vs_oracle():
    """n = 512 (the streaming soft top-k): a dense pair (float4 reads) and ragged pairs (row-strided
    reads) against the oracle."""
    g = torch.Generator().manual_seed(9)
    B, n = 3, 512
    n1s, n2s = [512, 480, 512], [512, 512, 437]
    ss = torch.rand(B, n, n, generator=g) ** 6
    for b in range(B):
        ss[b, n1s[b]:, :] = 0
        ss[b, :, n2s[b]:] = 0
    k = torch.tensor([120.5, 40.0, 300.0])
    ref = O.soft_topk(ss, k, n1s, n2s, 10, 0.01)
    out = ops.soft_topk_fwd(ss.to(DEV), _i32(n1s), _i32(n2s), k.to(DEV), 10, 0.01).cpu()
    assert (out - ref).abs().max() < 1e-4


def test_soft_topk_host_mapped_output():
    """The kernel's optional second output (pinned host memory, written over PCIe) equals the
    device output bit for bit, zero padding included."""
    g = torch.Generator().manual_seed(6)
    B, n = 3, 40
    ss = (torch.rand(B, n, n, generator=g) ** 4).to(DEV)
    n1, n2 = _i32([40, 31, 17]), _i32([40, 25, 33])
    k = torch.tensor([10.0, 12.5, 3.0]).to(DEV)
    host = torch.full((B, n, n), 7.0, pin_memory=True)
    out = ops.soft_topk_fwd(ss, n1, n2, k, 10, 0.01, out_host=host)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), host)
    assert (host[1, 31:, :] == 0).all() and (host[2, :, 33:] == 0).all()
    with pytest.raises(fpm._lib.FpmError):
        ops.soft_topk_fwd(ss, n1, n2, k, 10, 0.01, out_host=torch.empty(B, n, n))


# ---------------------------------------------------------------------------------------- top-k select
def test_topk_select_golden():
    z = np.load(os.path.join(GOLDEN, "hungarian_greedy.npz"))
    s = torch.from_numpy(z["s"])
    assign = ops.lsa_batch_host(s, torch.from_numpy(z["n1"]), torch.from_numpy(z["n2"]))
    perm = ops.topk_select(s.to(DEV), assign.to(DEV), torch.from_numpy(z["ks"]).to(DEV))
    np.testing.assert_array_equal(perm.cpu().numpy(), z["perm"])


@pytest.mark.parametrize("n1s,n2s,ks", [
    ((40, 31, 40), (40, 40, 22), (38.0, 30.5, 21.0)),     # k above the positive matches: zero-region fill
    ((256, 200), (256, 256), (120.5, 199.0)),
    ((64, 64), (64, 64), (7.0, 64.0)),
])
def test_topk_select_ranks_and_zero_region(n1s, n2s, ks):
    """fpm_topk_select (parallel ranks of the matches + ballot-counted zero-region fill) against the
    reference flow: prod = lsa * ds, stable descending argsort, greedy_perm (ngm.py:445-449,
    soft_topk.py:56-77), on matrices with many exact zeros and tied values."""
    g = torch.Generator().manual_seed(sum(n1s))
    B, n1max, n2max = len(n1s), max(n1s), max(n2s)
    ds = torch.rand(B, n1max, n2max, generator=g)
    ds = torch.where(torch.rand(B, n1max, n2max, generator=g) < 0.6, torch.zeros_like(ds), ds)
    ds = (ds * 8).round() / 8                                  # tied values
    for b in range(B):
        ds[b, n1s[b]:, :] = 0
        ds[b, :, n2s[b]:] = 0
    n1, n2 = torch.tensor(n1s, dtype=torch.int32), torch.tensor(n2s, dtype=torch.int32)
    assign = ops.lsa_batch_host(ds, n1, n2)
    kk = torch.tensor(ks)
    perm = ops.topk_select(ds.to(DEV), assign.to(DEV), kk.to(DEV)).cpu()
    lsa = O.hungarian(ds, n1s, n2s)
    prod = (lsa * ds).reshape(B, -1)
    top = torch.argsort(-prod, dim=-1, stable=True)
    ref = O.greedy_perm(torch.zeros(B, n1max, n2max), top, kk)
    assert torch.equal(perm, ref)


# ---------------------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("dt,tol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
def test_gemm_vs_torch(dt, tol):
    g = torch.Generator().manual_seed(3)
    M, N, K = 300, 200, 600
    A = torch.randn(M, K, generator=g)
    Bm = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    rows = torch.randint(0, M, (257,), generator=g)
    out = torch.empty(257, N, device=DEV)
    ops.gemm(A.to(DEV).to(dt), Bm.to(DEV).to(dt), 257, N, K, K, K, a_rows=rows.to(DEV).int(), epi=ops.EPI_RELU,
             bias=bias.to(DEV), out_f=out)
    ref = torch.relu(A.to(dt).float()[rows] @ Bm.to(dt).float().t() + bias)
    assert ((out.cpu() - ref).abs().max() / ref.abs().max()) < tol


@pytest.mark.parametrize("B,K,N", [(128, 1024, 768), (300, 1024, 768), (5, 1000, 300), (1, 17, 768)])
def test_coef_tanh_vs_float64_and_batch_independent(B, K, N):
    """Affinity coefficients tanh(g W^T + a) (affinity_layer.py:13): within 2e-6 of float64, and each
    row bit-identical whatever batch it is computed in (one fma chain per output)."""
    g = torch.Generator().manual_seed(11)
    gr = torch.nn.functional.normalize(torch.rand(B, K, generator=g), dim=1)
    wT = torch.randn(K, N, generator=g) * 0.05
    a = torch.randn(N, generator=g) * 0.1
    out = torch.empty(B, N, device=DEV)
    ops.coef_tanh(gr.to(DEV), wT.to(DEV), a.to(DEV), out)
    ref = torch.tanh(gr.double() @ wT.double() + a.double())
    assert float((out.cpu().double() - ref).abs().max()) < 2e-6
    one = torch.empty(1, N, device=DEV)
    ops.coef_tanh(gr[B - 1:].to(DEV), wT.to(DEV), a.to(DEV), one)
    assert torch.equal(one.cpu(), out.cpu()[B - 1:])


# ---------------------------------------------------------------------------------------- SplineConv
def test_spline_conv_vs_oracle(sd):
    pairs = synth.make_batch(11, 3, 40, n2=[40, 33, 21])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    net = fpm.Net(regression=True, backbone=False)
    net.load_state_dict(sd)
    out = net.run_gpu_stage(bt, keep_feats=True)
    for side, key in ((0, "feat0"), (1, "feat1")):
        nmax = bt.nmax[side]
        f = out[key].view(bt.B, nmax, -1).cpu()
        for b in range(bt.B):
            gph = pairs[b][side]
            ref = O.siamese_sconv(torch.from_numpy(gph["x"]), torch.from_numpy(gph["edge_index"]),
                                  torch.from_numpy(gph["pseudo"]), sd)
            assert (f[b, :gph["n"]] - ref).abs().max() < 2e-5
            assert f[b, gph["n"]:].abs().max() == 0 if gph["n"] < nmax else True


# ---------------------------------------------------------------------------------------- forward
def _compare_forward(pairs, sd, dtype="f32", tol=1e-4, regression=True):
    net = fpm.Net(regression=regression, backbone=False, dtype=dtype)
    net.load_state_dict(sd)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    res = net.run(bt)
    ref = O.forward(pairs, sd, regression=regression)
    d = {}
    for k in ("Kp", "s", "ss", "ds_mat", "k_prob", "cls_prob"):
        d[k] = float((res[k].float().cpu() - ref[k]).abs().max())
    d["perm_equal"] = bool(torch.equal(res["perm_mat"].cpu(), ref["perm_mat"]))
    return d


def test_forward_c1_parity(sd):
    """Config 1: single pair, 32 keypoints."""
    d = _compare_forward(synth.make_batch(1, 1, 32), sd)
    assert d["Kp"] < 1e-5 and d["s"] < 1e-4, d
    assert d["ss"] < 1e-4 and d["ds_mat"] < 1e-4 and d["k_prob"] < 1e-4, d
    assert d["perm_equal"], d
    assert d["cls_prob"] < 1e-4, d


@pytest.mark.parametrize("n,small", [(48, True), (72, False)])
def test_bf16_mode_small_graphs_take_fp32_spline(sd, n, small):
    """bf16 mode, batches whose padded box is at most Net.sc_f32_nmax (64) keypoints: the SplineConv
    products and the vertex affinity run in fp32, so s / ss equal the fp32 mode's bit for bit (the
    AFA-U stays bf16x3); above the threshold the bf16 products run (s differs, within the gate)."""
    pairs = synth.make_batch(61, 5, n, n2=[n - (b % 3) * 3 for b in range(5)])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    res = {}
    for dt in ("f32", "bf16"):
        net = fpm.Net(regression=True, backbone=False, dtype=dt)
        net.load_state_dict(sd)
        assert net._sc_f32(bt) == (dt == "f32" or small)
        res[dt] = net.run(bt)
    for k in ("s", "ss"):
        if small:
            assert torch.equal(res["f32"][k], res["bf16"][k]), k
        else:
            assert not torch.equal(res["f32"][k], res["bf16"][k]), k
            assert (res["f32"][k] - res["bf16"][k]).abs().max() < 1e-4, k


def test_forward_batch_parity(sd):
    d = _compare_forward(synth.make_batch(2, 4, 64), sd)
    assert d["ss"] < 1e-4 and d["ds_mat"] < 1e-4 and d["k_prob"] < 1e-4, d
    assert d["perm_equal"], d


def test_forward_ragged_parity(sd):
    """Ragged batch: padded p-space diagonal, dummy rows, transposed Sinkhorn, AFA-U padding."""
    d = _compare_forward(synth.make_batch(3, 3, [30, 24, 28], n2=[26, 30, 28]), sd)
    assert d["ss"] < 1e-4 and d["ds_mat"] < 1e-4 and d["k_prob"] < 1e-4, d
    assert d["perm_equal"], d


def test_forward_no_regression_parity(sd):
    d = _compare_forward(synth.make_batch(4, 2, 48), sd, regression=False)
    assert d["ss"] < 1e-4 and d["ds_mat"] < 1e-4, d
    assert d["perm_equal"], d


def _run_and_ref(pairs, sd, dtypes=("f32",), regression=True, bt=None, afau=None):
    """The device forward in each compute mode and the oracle on the same pairs (``afau``: the
    AFA-U mode of the bf16 runs, default the library's)."""
    ref = O.forward(pairs, sd, regression=regression)
    outs = {}
    for dt in dtypes:
        net = fpm.Net(regression=regression, backbone=False, dtype=dt, afau=afau)
        net.load_state_dict(sd)
        outs[dt] = net.run(bt if bt is not None else DeviceBatch.from_pairs(pairs, DEV))
    return outs, ref


def _perm_gate(res, ref, pairs, name):
    """perm_mat against the oracle, pair by pair (oracle.compare): every pair identical or differing
    only by a (near-)tie or a k* rounding-boundary crossing; the classes are recorded."""
    n1 = [p[0]["n"] for p in pairs]
    n2 = [p[1]["n"] for p in pairs]
    bf16 = "bf16" in name
    # k* rounding crossings are judged against the mode's own k_prob tolerance
    rep = O.compare.perm_report(res, ref, n1, n2, reduced_precision=bf16,
                                k_tol=2.0 * BF16_MEASURED["k_prob"] if bf16 else 1e-4)
    _record(name, {k: v for k, v in rep.items()})
    assert rep["counts"]["mismatch"] == 0, rep
    return rep


def test_forward_n256_parity(sd):
    """Benchmark graph size (C3's n=256), 16 pairs, fp32 mode vs the oracle: ss / ds_mat / k_prob
    within 1e-4 and every pair's perm_mat identical or explained (tie / k* rounding; the identical
    fraction is recorded).  The bf16 headline mode on the same pairs gets the bf16 gates."""
    pairs = synth.make_batch(5, 16, 256)
    outs, ref = _run_and_ref(pairs, sd, ("f32", "bf16"), afau="bf16s")
    res = outs["f32"]
    d = {k: float((res[k].float().cpu() - ref[k]).abs().max()) for k in ("ss", "ds_mat", "k_prob", "cls_prob")}
    assert d["ss"] < 1e-4 and d["ds_mat"] < 1e-4 and d["k_prob"] < 1e-4 and d["cls_prob"] < 1e-4, d
    _perm_gate(res, ref, pairs, "perm_report_n256_f32")
    db = fidelity_stats(outs["bf16"], ref)
    _record("bf16_fidelity_c3_16", db)
    _bf16_gate(db)
    _perm_gate(outs["bf16"], ref, pairs, "perm_report_n256_bf16")


def test_forward_c2_parity(sd):
    """SURVEY config C2 (n = 128, fp32 mode) vs the oracle: 1e-4 on ss / ds_mat / k_prob and
    cls_prob, perm_mat explained pair by pair (ngm.py:479-487)."""
    pairs = synth.make_batch(13, 6, 128)
    outs, ref = _run_and_ref(pairs, sd, ("f32",))
    res = outs["f32"]
    d = {k: float((res[k].float().cpu() - ref[k]).abs().max()) for k in ("Kp", "ss", "ds_mat", "k_prob", "cls_prob")}
    _record("c2_parity", d)
    assert d["Kp"] < 1e-5 and d["ss"] < 1e-4 and d["ds_mat"] < 1e-4 and d["k_prob"] < 1e-4, d
    assert d["cls_prob"] < 1e-4, d
    _perm_gate(res, ref, pairs, "perm_report_c2")


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_forward_c4_probe_gallery_vs_oracle(sd, dtype):
    """SURVEY config C4 (1 probe x gallery, n = 128; evaluate_binary_classifier.py:97): the
    probe-shared batch (the probe's SplineConv computed once and broadcast) against the oracle
    run on the expanded (probe, gallery_g) pairs: fp32 at 1e-4, bf16 under the bf16 gates."""
    probe = synth.make_graph(17, 0, 0, 128)
    gallery = [synth.make_graph(17, 1 + g, 1, 128 - (g % 3) * 5) for g in range(6)]
    pairs = [(probe, g) for g in gallery]
    bt = DeviceBatch.from_probe_gallery(probe, gallery, DEV)
    outs, ref = _run_and_ref(pairs, sd, (dtype,), bt=bt, afau="bf16s")
    res = outs[dtype]
    if dtype == "f32":
        d = {k: float((res[k].float().cpu() - ref[k]).abs().max()) for k in ("ss", "ds_mat", "k_prob", "cls_prob")}
        _record("c4_parity_f32", d)
        assert d["ss"] < 1e-4 and d["ds_mat"] < 1e-4 and d["k_prob"] < 1e-4 and d["cls_prob"] < 1e-4, d
    else:
        d = fidelity_stats(res, ref)
        _record("c4_fidelity_bf16", d)
        _bf16_gate(d)
    _perm_gate(res, ref, pairs, "perm_report_c4_" + dtype)


def _fidelity(pairs, sd, dtype="bf16", afau="bf16s"):
    """Deviation of a reduced-precision forward from the fp32 oracle on the same pairs: max|d| per
    output, and perm_mat agreement (all entries, the oracle's matches kept, pairs identical).  The
    default AFA-U mode of dtype bf16 (bf16x3) is held to the 1e-4 gate by test_gated_mode_*; these
    fidelity tests cover the cheaper bf16s AFA-U variant under the reported (looser) bounds."""
    net = fpm.Net(regression=True, dtype=dtype, backbone=False, afau=afau)
    net.load_state_dict(sd)
    res = net.run(DeviceBatch.from_pairs(pairs, DEV))
    ref = O.forward(pairs, sd, regression=True)
    return fidelity_stats(res, ref), res, ref


def fidelity_stats(res, ref):
    d = {k: float((res[k].float().cpu() - ref[k]).abs().max()) for k in ("Kp", "s", "ss", "ds_mat", "k_prob",
                                                                           "cls_prob")}
    P, R = res["perm_mat"].cpu(), ref["perm_mat"]
    d["perm_entries_agree"] = float((P == R).float().mean())
    d["perm_matches_kept"] = float((P * R).sum() / R.sum().clamp(min=1))
    d["perm_pairs_identical"] = float(np.mean([torch.equal(P[b], R[b]) for b in range(P.shape[0])]))
    # same count and the oracle's ds_mat values at the picks equal: differs only among (near-)ties
    d["perm_pairs_tie_equivalent"] = float(np.mean([
        int((P[b] > 0).sum()) == int((R[b] > 0).sum()) and
        bool(((torch.sort(ref["ds_mat"][b][P[b] > 0]).values - torch.sort(ref["ds_mat"][b][R[b] > 0]).values).abs()
              .max() <= 1e-5) if int((R[b] > 0).sum()) else True) for b in range(P.shape[0])]))
    return d


def _record(name, d):
    import json
    out = os.path.join(REPO, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, name + ".json"), "w") as f:
        json.dump(d, f, indent=1)
    print(name, d)


# bf16 mode vs the fp32 oracle: the largest deviations measured on the box by the fidelity tests
# (round 2: n = 128 / 256 / 512 -> gpurun_out/bf16_fidelity_*.json) and the bench's 8-pair C3 sample
BF16_MEASURED = {"Kp": 1.4e-5, "ss": 1.4e-6, "ds_mat": 4.5e-6, "k_prob": 8.7e-4, "cls_prob": 2.7e-5}
# (round-3 final tree: largest values over the C2 / C3 / C3-16 / C4 / C5 fidelity records and the bench
# sample -- Kp 1.36e-5, ss 1.40e-6, ds_mat 4.44e-6 (C4), k_prob 7.7e-4 (bench), cls_prob 2.7e-5)


def _bf16_gate(d):
    """Bounds for the bf16 throughput mode against the fp32 oracle (reported, with
    these gates): 2x the largest deviation measured (BF16_MEASURED), and every pair's perm_mat
    identical or tie-equivalent (a different pick among (near-)tied soft top-k entries) -- a k*
    rounding crossing is judged by _perm_gate, which classifies pair by pair."""
    for k, v in BF16_MEASURED.items():
        assert d[k] < 2.0 * v, (k, d[k], 2.0 * v, d)
    assert d["perm_matches_kept"] >= 0.98, d


def test_forward_bf16_fidelity_n128(sd):
    """bf16 MFMA mode vs the fp32 oracle at n=128 (C2 size)."""
    pairs = synth.make_batch(6, 2, 128)
    d, res, ref = _fidelity(pairs, sd)
    _record("bf16_fidelity_n128", d)
    _bf16_gate(d)
    _perm_gate(res, ref, pairs, "perm_report_bf16_n128")


def test_forward_bf16_fidelity_c3(sd):
    """SURVEY §8(d) parity gate for the headline mode: bf16 at C3's graph size (n=256, B=4) vs the
    fp32 oracle, max|d| on ss / ds_mat / k_prob / cls_prob and perm_mat agreement, recorded and bounded."""
    pairs = synth.make_batch(61, 4, 256)
    d, res, ref = _fidelity(pairs, sd)
    _record("bf16_fidelity_c3", d)
    _bf16_gate(d)
    _perm_gate(res, ref, pairs, "perm_report_bf16_c3")


@pytest.mark.slow
def test_forward_bf16_fidelity_c5(sd):
    """The same gate at C5's graph size (n=512, B=1)."""
    pairs = synth.make_batch(62, 1, 512)
    d, res, ref = _fidelity(pairs, sd)
    _record("bf16_fidelity_c5", d)
    _bf16_gate(d)
    _perm_gate(res, ref, pairs, "perm_report_bf16_c5")


def test_forward_data_dict_surface(sd):
    """Reference-shaped data_dict in, reference keys out (ngm.py:479-487)."""
    pairs = synth.make_batch(8, 2, 24, n2=[24, 20])
    B = 2

    class G:
        pass
    dd = {"ns": [torch.tensor([p[0]["n"] for p in pairs]), torch.tensor([p[1]["n"] for p in pairs])],
          "pyg_graphs": [], "node_features": [], "global_features": []}
    for side in range(2):
        g = G()
        offs = np.cumsum([0] + [p[side]["n"] for p in pairs])
        g.edge_index = torch.from_numpy(np.concatenate([p[side]["edge_index"] + offs[b] for b, p in enumerate(pairs)], 1))
        g.edge_attr = torch.from_numpy(np.concatenate([p[side]["pseudo"] for p in pairs]))
        g.ptr = torch.from_numpy(offs)
        dd["pyg_graphs"].append(g)
        dd["node_features"].append(torch.from_numpy(np.concatenate([p[side]["x"] for p in pairs])))
        dd["global_features"].append(torch.from_numpy(np.stack([p[side]["w"] for p in pairs])))
    gt = torch.zeros(B, 24, 24)
    for b in range(B):
        m = min(pairs[b][0]["n"], pairs[b][1]["n"])
        gt[b, range(m), range(m)] = 1
    dd["gt_perm_mat"] = gt
    dd["label"] = torch.tensor([1.0, 0.0])
    net = fpm.Net(regression=True, backbone=False)
    net.load_state_dict(sd)
    out = net(dd)
    for k in ("ds_mat", "perm_mat", "ks_loss", "ks_error", "cls_loss", "cls_prob", "k_prob"):
        assert k in out
    ref = O.forward(pairs, sd, gt_perm=gt, labels=torch.tensor([1.0, 0.0]))
    assert (out["ds_mat"].cpu() - ref["ds_mat"]).abs().max() < 1e-4
    assert abs(float(out["ks_loss"]) - float(ref["ks_loss"])) < 1e-3
    assert abs(float(out["cls_loss"]) - float(ref["cls_loss"])) < 1e-4


@pytest.mark.parametrize("n", [48, 96])
def test_chunked_pipeline_bitwise(sd, n):
    """Pipelined sub-batches (host LSA of chunk c overlapping GPU work of c+1) give bit-identical
    outputs to the single-chunk forward; the same property makes pair-sharding across GPUs exact.
    n = 48: the fp64 k chain; n = 96: the fp32 GNN / Sinkhorn kernels."""
    d = n - 48
    pairs = synth.make_batch(9, 7, n, n2=[x + d for x in (48, 40, 44, 48, 30, 48, 47)])
    net = fpm.Net(regression=True, backbone=False, dtype="bf16")
    net.load_state_dict(sd)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    a = net.run(bt, chunks=1)
    b = net.run(bt, chunks=3)
    for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert torch.equal(a[k], b[k]), k
    # a shard computed alone (as another rank would) equals its slice of the full batch
    sub = DeviceBatch.from_pairs(pairs[2:5], DEV)
    sub.nmax = list(bt.nmax)
    c = net.run(sub, chunks=1)
    for k in ("ds_mat", "perm_mat", "k_prob"):
        assert torch.equal(c[k], a[k][2:5]), k


def test_spline_plans_multi_equal_per_chunk_plans(sd):
    """Every chunk's spline plans built by one launch per plan kernel (fpm_spline_plan_multi) equal
    the per-chunk plans: dst CSR arrays identical, and the forward through each plan identical."""
    pairs = synth.make_batch(27, 9, [48, 40, 44, 48, 30, 48, 47, 41, 48], n2=[48, 47, 40, 30, 48, 44, 48, 48, 39])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    parts = bt.split(3, 1)
    for side in range(2):
        multi = ops.spline_plans_multi(parts, side, bt.nmax[side])
        assert multi is not None and len(multi) == len(parts)
        for p, m in zip(parts, multi):
            one = ops.spline_plan(p.src[side], p.dst[side], p.pseudo[side], p.B * p.nmax[side], p.nmax[side],
                                  p.max_graph_edges(side))
            nn = p.B * p.nmax[side]
            ca, cb = ops.plan_csr(one, p.E[side], nn), ops.plan_csr(m, p.E[side], nn)
            for pa, pb, cnt in ((ca[0], cb[0], nn + 1), (ca[1], cb[1], p.E[side])):
                torch.cuda.synchronize()
                assert torch.equal(_view_i32(pa, cnt), _view_i32(pb, cnt))
    net = fpm.Net(regression=True, backbone=False, dtype="bf16", chunks=3)
    net.load_state_dict(sd)
    a = net.run(bt)
    b = net.run(bt, chunks=1)
    for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert torch.equal(a[k], b[k]), k


@pytest.mark.parametrize("chunks", [1, 3])
def test_prologue_graph_bitwise_equals_eager(sd, chunks):
    """The eager forward's prologue replayed from a HIP graph (FPM_PROLOGUE_GRAPH=2 here: every
    forward; the default 1 replays it for one-chunk forwards: the coefficients, casts, AFA-U column
    block and every chunk's spline plans) is bit-identical to launching it eagerly: on the capturing forward, on replays, and
    after another batch made it recapture."""
    pairs = synth.make_batch(31, 11, [48, 40, 44, 48, 30, 48, 47, 41, 48, 36, 45],
                             n2=[48, 47, 40, 30, 48, 44, 48, 48, 39, 48, 42])
    other = synth.make_batch(32, 5, 40)
    bt, bo = DeviceBatch.from_pairs(pairs, DEV), DeviceBatch.from_pairs(other, DEV)
    keys = ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob")
    runs = {}
    for pg in (False, True):
        net = fpm.Net(regression=True, backbone=False, dtype="bf16", chunks=chunks)
        net.load_state_dict(sd)
        net.prologue_graph = 2 if pg else 0
        r = [{k: v.clone() for k, v in net.run(bt).items() if k in keys} for _ in range(2)]
        ro = {k: v.clone() for k, v in net.run(bo).items() if k in keys}
        r.append({k: v.clone() for k, v in net.run(bt).items() if k in keys})
        assert (net._pgstate is not None) == pg
        runs[pg] = (r, ro)
    for i in range(3):
        for k in keys:
            assert torch.equal(runs[False][0][i][k], runs[True][0][i][k]), (i, k)
    for k in keys:
        assert torch.equal(runs[False][1][k], runs[True][1][k]), k


def _view_i32(ptr, n):
    """A device int32 array at a raw pointer, as a torch tensor (copy)."""
    out = torch.empty(n, dtype=torch.int32, device=DEV)
    import ctypes
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipMemcpy(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(4 * n), 3)
    return out


@pytest.mark.parametrize("dtype,regression,d", [("bf16", True, 0), ("f32", False, 0), ("bf16", True, 40)])
def test_graph_replay_bitwise_equals_eager(sd, dtype, regression, d):
    """Multi-chunk forwards replay HIP graphs captured on the batch's first forward (prologue, and
    per chunk its plans and GPU stage): bit-identical to the eager launches on a ragged batch, on
    the capturing forward and on replays; the returned reference outputs are fresh tensors.
    d = 40: boxes of 88 keypoints (the fp32 GNN / Sinkhorn kernels; below 64 the fp64 k chain)."""
    pairs = synth.make_batch(23, 11, [x + d for x in (48, 40, 44, 48, 30, 48, 47, 41, 48, 36, 45)],
                             n2=[x + d for x in (48, 47, 40, 30, 48, 44, 48, 48, 39, 48, 42)])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    runs = {}
    for graphs in (False, True):
        net = fpm.Net(regression=regression, backbone=False, dtype=dtype, chunks=3)
        net.load_state_dict(sd)
        net.use_graphs = graphs
        r = [net.run(bt) for _ in range(3)]
        assert net.last_timing["graphs"] == graphs and net.last_timing["chunks"] > 1
        runs[graphs] = r
    for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob", "lsa"):
        for r in runs[True]:
            assert torch.equal(runs[False][0][k], r[k]), k
    a, b = runs[True][0], runs[True][1]
    assert a["ds_mat"].data_ptr() != b["ds_mat"].data_ptr() and a["perm_mat"].data_ptr() != b["perm_mat"].data_ptr()


# ---------------------------------------------------------------------------------------- Ke, Gconv
def test_edge_affinity_ke(sd):
    """Optional quadratic affinity (ngm.py:282-289) vs the oracle, ragged edge counts."""
    pairs = synth.make_batch(12, 3, [20, 31, 26], n2=[24, 18, 30])
    net = fpm.Net(regression=True, backbone=False, compute_ke=True)
    net.load_state_dict(sd)
    res = net.run(DeviceBatch.from_pairs(pairs, DEV))
    ref = O.forward(pairs, sd, regression=True, compute_ke=True)
    Ke = res["Ke"].cpu()
    for b in range(3):
        e1, e2 = ref["Ke"][b].shape
        assert (Ke[b, :e1, :e2] - ref["Ke"][b]).abs().max() < 1e-5
        assert Ke[b, e1:].abs().max() == 0 if e1 < Ke.shape[1] else True
        assert Ke[b, :, e2:].abs().max() == 0 if e2 < Ke.shape[2] else True
    assert (res["ds_mat"].cpu() - ref["ds_mat"]).abs().max() < 1e-4


def test_gconv_golden():
    from fpm.gconv import Gconv
    z = np.load(os.path.join(GOLDEN, "gconv.npz"))
    gc = Gconv(6, 5)
    with torch.no_grad():
        gc.a_fc.weight.copy_(torch.from_numpy(z["a_w"]))
        gc.a_fc.bias.copy_(torch.from_numpy(z["a_b"]))
        gc.u_fc.weight.copy_(torch.from_numpy(z["u_w"]))
        gc.u_fc.bias.copy_(torch.from_numpy(z["u_b"]))
    A, x = torch.from_numpy(z["A"]), torch.from_numpy(z["x"])
    y = gc(A.to(DEV), x.to(DEV)).cpu()
    np.testing.assert_allclose(y.numpy(), z["y"], atol=1e-5, rtol=0)
    y2 = gc(A.to(DEV), x.to(DEV), norm=False).cpu()
    ref = O.gconv(A, x, *(torch.from_numpy(z[k]) for k in ("a_w", "a_b", "u_w", "u_b")), norm=False)
    assert (y2 - ref).abs().max() < 1e-5


@pytest.mark.parametrize("C,layer", [(1, 0), (17, 1)])
def test_gnn_layer_vs_oracle(sd, C, layer):
    """Kronecker GNN layer (gnn.hip) on a ragged batch: x1 (Xout channels 0..15) and the
    classifier logit z against the oracle's factorised aggregation + MLPs."""
    import torch.nn.functional as F
    from fpm import synth
    n1s, n2s = [40, 33, 25], [40, 38, 20]
    B, nm = 3, 40
    pairs = synth.make_batch(11, B, n1s, n2s)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    plans = [ops.spline_plan(bt.src[s], bt.dst[s], bt.pseudo[s], B * nm, nm) for s in range(2)]
    csr = [ops.plan_csr(plans[s], bt.E[s], B * nm) for s in range(2)]
    net = fpm.Net(regression=True, backbone=False, dtype="f32", seed=7)
    wp = net.packed(DEV)
    g = torch.Generator().manual_seed(C)
    X = torch.randn(B, C, nm, nm, generator=g)                 # [b][c][j (graph 2)][i (graph 1)]
    Xn = torch.full((B, 17, nm, nm), 5.0, device=DEV)
    z = torch.full((B, nm, nm), 5.0, device=DEV)
    ops.gnn_layer(X.to(DEV), C, B, nm, nm, csr[0], csr[1], bt.n1, bt.n2, wp["gnn%d" % layer], Xn, z)
    torch.cuda.synchronize()
    Xn, z = Xn.cpu(), z.cpu()
    pre = "gnn_layer_%d" % layer
    w = lambda k: sd[pre + k].float()
    for b in range(B):
        ei1 = torch.as_tensor(pairs[b][0]["edge_index"])
        ei2 = torch.as_tensor(pairs[b][1]["edge_index"])
        x = X[b].reshape(C, nm * nm).t()                       # p = j * nm + i
        agg = O.pattern_mean_factorized(x, ei1, ei2, nm, nm, n1s[b], n2s[b])
        x1 = F.linear(agg, w(".conv2.lin_l.weight"), w(".conv2.lin_l.bias")) + F.linear(x, w(".conv2.lin_r.weight"))
        h = F.relu(F.linear(x, w(".n_self_func.0.weight"), w(".n_self_func.0.bias")))
        x1 = x1 + F.relu(F.linear(h, w(".n_self_func.2.weight"), w(".n_self_func.2.bias")))
        zr = F.linear(x1, w(".classifier.weight"), w(".classifier.bias"))[:, 0]
        assert (Xn[b, :16].reshape(16, -1).t() - x1).abs().max() < 1e-4
        assert (z[b].reshape(-1) - zr).abs().max() < 1e-4


@pytest.mark.parametrize("M,N,K,batch,epi,f32out,gather", [
    (1000, 600, 256, 1, 1, True, False),      # AFA-U W2 / Wc shape: N tail, 256x128 tiles
    (1000, 256, 640, 1, 1, False, False),     # FFN W1 (zero-padded K), bf16 out
    (2048, 768, 768, 1, 0, False, True),      # gathered rows, 256x256 tiles
    (600, 512, 128, 3, 0, True, False),       # batched
])
def test_gemm_big_vs_torch(M, N, K, batch, epi, f32out, gather):
    """The 256-row LDS-DMA bf16 kernel (gemm_big.h) through fpm_gemm: bias, ReLU, fp32/bf16 out,
    row gather, batch strides, N tails."""
    g = torch.Generator().manual_seed(M + N)
    A = torch.randn(batch, M + 17, K, generator=g).to(torch.bfloat16)
    Bm = (torch.randn(batch, N, K, generator=g) * 0.1).to(torch.bfloat16)
    bias = torch.randn(N, generator=g)
    rows = torch.randint(0, M + 17, (M,), generator=g) if gather else None
    Ad, Bd = A.to(DEV), Bm.to(DEV)
    out = torch.empty(batch, M, N, device=DEV, dtype=torch.float32 if f32out else torch.bfloat16)
    kw = dict(out_f=out) if f32out else dict(out_t=out)
    ops.gemm(Ad, Bd, M, N, K, K, K, batch=batch, sA=(M + 17) * K, sB=N * K, sC=M * N,
             a_rows=rows.to(DEV).int() if gather else None, epi=epi, bias=bias.to(DEV), **kw)
    Af = A.float()[:, rows] if gather else A.float()[:, :M]
    ref = Af @ Bm.float().transpose(1, 2) + bias
    if epi == 1:
        ref = torch.relu(ref)
    tol = 2e-3 if f32out else 1e-2
    assert ((out.float().cpu() - ref).abs().max() / ref.abs().max()) < tol


@pytest.mark.parametrize("M,N,K,batch,epi,f32out,gather", [
    (46080 + 37, 768, 768, 1, 0, False, True),   # SplineConv product shape: gathered rows, row tail
    (40000, 512, 128, 1, 1, True, False),        # 2 K-tiles (shortest pipeline), ReLU, fp32 out
    (33000, 1024, 192, 1, 0, False, False),      # 3 K-tiles
    (256, 256, 256, 520, 3, True, False),        # batched affinity epilogue
])
def test_gemm_phase_bit_identical(M, N, K, batch, epi, f32out, gather):
    """The phase-pipelined 256x256 kernel (gemm_phase.h) against the two-stage kernel: same
    accumulation order, so bit-identical outputs; and both against torch."""
    g = torch.Generator().manual_seed(M + K)
    A = (torch.randn(batch, M + 17, K, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    Bm = (torch.randn(batch, N, K, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV) if epi != 3 else None
    rows = torch.randint(0, M + 17, (M,), generator=g).to(DEV).int() if gather else None
    n1 = torch.randint(1, 257, (batch,), generator=g).int().to(DEV) if epi == 3 else None
    n2 = torch.randint(1, 257, (batch,), generator=g).int().to(DEV) if epi == 3 else None
    outs = []
    for phase in (1, 0):
        prev = ops.set_tuning("gemm_phase", phase)
        try:
            out = torch.full((batch, M, N), 3.0, device=DEV, dtype=torch.float32 if f32out else torch.bfloat16)
            kw = dict(out_f=out) if f32out else dict(out_t=out)
            ops.gemm(A, Bm, M, N, K, K, K, batch=batch, sA=(M + 17) * K, sB=N * K, sC=M * N, a_rows=rows,
                     epi=epi, bias=bias, n1=n1, n2=n2, **kw)
            torch.cuda.synchronize()
        finally:
            ops.set_tuning("gemm_phase", prev)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])
    Af = A.float()[:, rows.long()] if gather else A.float()[:, :M]
    ref = Af @ Bm.float().transpose(1, 2)
    if bias is not None:
        ref = ref + bias
    if epi == 1:
        ref = torch.relu(ref)
    if epi == 3:
        ref = torch.nn.functional.softplus(ref) - 0.5
        r = torch.arange(M, device=DEV)[None, :, None] < n2[:, None, None]
        c = torch.arange(N, device=DEV)[None, None, :] < n1[:, None, None]
        ref = torch.where(r & c, ref, torch.zeros_like(ref))
    tol = 2e-3 if f32out else 1e-2
    assert ((outs[0].float() - ref).abs().max() / ref.abs().max()).item() < tol


# ---------------------------------------------------------------------------------------- large n (C5)
def test_sinkhorn_stream_vs_oracle():
    """n > 256: the L2-streaming Sinkhorn (dummy rows, transposed pair, strided views)."""
    g = torch.Generator().manual_seed(21)
    n1s, n2s = (512, 300, 512), (512, 512, 400)
    B, n1max, n2max = 3, 512, 512
    s = torch.randn(B, n1max, n2max, generator=g) * 0.3
    ref = O.pygm_sinkhorn(s.double(), n1s, n2s, dummy_row=True, max_iter=10, tau=0.01)
    out = ops.sinkhorn(s.to(DEV), _i32(n1s), _i32(n2s), 10, 0.01, True).cpu()
    assert (out.double() - ref).abs().max() < 1e-4
    sT = s.transpose(1, 2).contiguous().to(DEV).transpose(1, 2)
    o2 = torch.zeros(B, n2max, n1max, device=DEV).transpose(1, 2)
    ops.sinkhorn(sT, _i32(n1s), _i32(n2s), 10, 0.01, True, out=o2)
    assert (o2.cpu().double() - ref).abs().max() < 1e-4


@pytest.mark.parametrize("n1s,n2s,tau", [
    ((437, 512, 511), (512, 301, 509), 0.01),        # valid widths % 4 != 0: scalar shifted-sum paths
    ((300, 437), (437, 300), 0.0005),                # very small tau: sums leave [2^-30, 2^30] -> fallback
])
def test_sinkhorn_stream_ragged_vs_oracle(n1s, n2s, tau):
    """Streaming Sinkhorn on ragged widths that are not multiples of 4 (dummy rows, transposed
    pairs) and at a temperature that drives the shifted sums out of range (max-shifted fallback)."""
    g = torch.Generator().manual_seed(23 + len(n1s))
    B, n1max, n2max = len(n1s), max(n1s), max(n2s)
    s = torch.randn(B, n1max, n2max, generator=g) * 0.3
    ref = O.pygm_sinkhorn(s.double(), n1s, n2s, dummy_row=True, max_iter=10, tau=tau)
    out = ops.sinkhorn(s.to(DEV), _i32(n1s), _i32(n2s), 10, tau, True).cpu()
    assert (out.double() - ref).abs().max() < 1e-4


@pytest.mark.parametrize("tau", [0.01, 0.0005])
def test_sinkhorn_stream_split_vs_oracle(tau):
    """Boxes over 256 through ops.sinkhorn: square / dummy-free pairs run on FPM_SK_SPLIT workgroups
    that exchange partial column sums (tau 0.0005 drives the shifted sums out of range: the exact
    (max, sum) exchange); pairs with dummy rows run whole on one workgroup of the same launch.  Both
    layouts; deterministic; a pair's result does not depend on the batch; and within 1e-5 of the
    one-workgroup form (fpm_sinkhorn_log_fwd without a workspace)."""
    g = torch.Generator().manual_seed(31)
    n1s, n2s = (512, 400, 300, 512, 260, 256, 512), (512, 400, 512, 300, 260, 256, 497)
    B, n1max, n2max = len(n1s), 512, 512
    s = torch.randn(B, n1max, n2max, generator=g) * 0.3
    # fp32 entries s / tau reach ~3e3 at tau = 0.0005: ~2e-4 of rounding in the log domain for any
    # fp32 form (the one-workgroup kernel measures 1.06e-4 on the transposed layout); 1e-4 at 0.01
    tol = 1e-4 if tau >= 0.01 else 2e-4
    ref = O.pygm_sinkhorn(s.double(), n1s, n2s, dummy_row=True, max_iter=10, tau=tau)
    sd, n1d, n2d = s.to(DEV), _i32(n1s), _i32(n2s)
    out = ops.sinkhorn(sd, n1d, n2d, 10, tau, True)
    assert (out.cpu().double() - ref).abs().max() < tol
    assert torch.equal(out, ops.sinkhorn(sd, n1d, n2d, 10, tau, True))
    solo = ops.sinkhorn(sd[:2].contiguous(), n1d[:2].contiguous(), n2d[:2].contiguous(), 10, tau, True)
    assert torch.equal(solo, out[:2])
    sT = s.transpose(1, 2).contiguous().to(DEV).transpose(1, 2)
    o2 = torch.zeros(B, n2max, n1max, device=DEV).transpose(1, 2)
    ops.sinkhorn(sT, n1d, n2d, 10, tau, True, out=o2)
    assert (o2.cpu().double() - ref).abs().max() < tol
    one = torch.empty_like(out)
    _lib.call("fpm_sinkhorn_log_fwd", ops._p(sd), *sd.stride(), ops._p(one), *one.stride(), ops._p(n1d),
              ops._p(n2d), B, n1max, n2max, 10, float(tau), 1, ops._stream(sd))
    torch.cuda.synchronize()
    assert (one - out).abs().max().item() < 1e-5
    # dummy_row=False: rectangular pairs have no dummy rows, so they split as well
    ref_nd = O.pygm_sinkhorn(s.double(), n1s, n2s, dummy_row=False, max_iter=10, tau=tau)
    out_nd = ops.sinkhorn(sd, n1d, n2d, 10, tau, False)
    assert (out_nd.cpu().double() - ref_nd).abs().max() < tol


def test_sinkhorn_max_box_and_empty_batch():
    """The largest supported box (2048 x 2048, SK_MAXN) through both streaming forms (the split one
    via ops.sinkhorn, one workgroup per pair via fpm_sinkhorn_log_fwd) against the fp64 oracle, a
    ragged pair with dummy rows beside a square one; and B = 0 launches nothing."""
    g = torch.Generator().manual_seed(37)
    n1s, n2s = (2048, 1500), (2048, 2048)
    B, nm = 2, 2048
    s = torch.randn(B, nm, nm, generator=g) * 0.3
    ref = O.pygm_sinkhorn(s.double(), n1s, n2s, dummy_row=True, max_iter=10, tau=0.01)
    sd, n1d, n2d = s.to(DEV), _i32(n1s), _i32(n2s)
    out = ops.sinkhorn(sd, n1d, n2d, 10, 0.01, True)
    assert (out.cpu().double() - ref).abs().max() < 1e-4
    one = torch.empty_like(out)
    _lib.call("fpm_sinkhorn_log_fwd", ops._p(sd), *sd.stride(), ops._p(one), *one.stride(), ops._p(n1d),
              ops._p(n2d), B, nm, nm, 10, 0.01, 1, ops._stream(sd))
    torch.cuda.synchronize()
    assert (one.cpu().double() - ref).abs().max() < 1e-4
    e = torch.empty(0, 512, 512, device=DEV)
    z = torch.empty(0, dtype=torch.int32, device=DEV)
    assert ops.sinkhorn(e, z, z, 10, 0.01, True).shape == (0, 512, 512)
    assert ops.soft_topk_fwd(e, z, z, torch.empty(0, device=DEV), 10, 0.01).shape == (0, 512, 512)


def test_soft_topk_large_box_vs_oracle():
    """Soft top-k on a 1024 x 1024 pair (the streaming form, 16 M-entry passes) and a ragged
    1024 x 700 pair in the same box, against the oracle incl. its while loop."""
    g = torch.Generator().manual_seed(43)
    n1s, n2s = [1024, 1024], [1024, 700]
    ss = torch.rand(2, 1024, 1024, generator=g) ** 8
    ss[1, :, 700:] = 0
    k = torch.tensor([600.5, 350.0])
    ref = O.soft_topk(ss, k, n1s, n2s, 10, 0.01)
    out = ops.soft_topk_fwd(ss.to(DEV), _i32(n1s), _i32(n2s), k.to(DEV), 10, 0.01).cpu()
    assert (out - ref).abs().max() < 1e-4


def test_gnn_block_order_bit_identical(sd):
    """Boxes over 256 run the GNN layers' (pair, graph-2 node) workgroups in Hilbert order of the
    keypoints (DeviceBatch.ord2, a schedule only): the forward is bit-identical to the identity order,
    and the batch carries a permutation per pair (padding slots last, in index order)."""
    from fpm.batch import hilbert_order
    pairs = synth.make_batch(41, 3, [300, 290, 270], [280, 300, 300])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    assert bt.ord2 is not None and tuple(bt.ord2.shape) == (3, 300)
    o = bt.ord2.cpu()
    for b, p in enumerate(pairs):
        assert sorted(o[b].tolist()) == list(range(300))
        assert o[b, p[1]["n"]:].tolist() == list(range(p[1]["n"], 300))
    assert torch.equal(hilbert_order(torch.zeros(1, 4, 2), [4], 4).cpu(), torch.arange(4, dtype=torch.int32)[None])
    net = fpm.Net(regression=True, backbone=False, dtype="bf16")
    net.load_state_dict(sd)
    r1 = net.run(bt, chunks=1)
    torch.cuda.synchronize()
    bt2 = DeviceBatch.from_pairs(pairs, DEV)
    bt2.ord2 = None
    r2 = net.run(bt2, chunks=1)
    torch.cuda.synchronize()
    for k in ("s", "ss", "ds_mat", "k_prob", "perm_mat"):
        assert torch.equal(r1[k], r2[k]), k


def test_soft_topk_stream_vs_oracle():
    g = torch.Generator().manual_seed(22)
    B, n = 2, 512
    ss = torch.rand(B, n, n, generator=g) ** 6
    k = torch.tensor([100.5, 400.0])
    ref = O.soft_topk(ss, k, [n] * B, [n] * B, 10, 0.01)
    out = ops.soft_topk_fwd(ss.to(DEV), _i32([n] * B), _i32([n] * B), k.to(DEV), 10, 0.01).cpu()
    assert (out - ref).abs().max() < 1e-4


@pytest.mark.slow
def test_forward_n512_parity(sd):
    """C5 graph size (n = 512) end to end at a batch the CPU oracle finishes in tens of seconds."""
    d = _compare_forward(synth.make_batch(31, 1, 512), sd)
    assert d["ss"] < 1e-4 and d["ds_mat"] < 1e-4 and d["k_prob"] < 1e-4, d
    assert d["perm_equal"], d


@pytest.mark.slow
def test_forward_univ_size_cap(sd):
    """The largest box the reference accepts (UNIV_SIZE = 600, ngm.py:387-389) end to end against
    the oracle, a ragged partner in the same batch; one keypoint more is refused like the reference's
    assertion."""
    pairs = synth.make_batch(33, 1, [600], [571])
    d = _compare_forward(pairs, sd)
    assert d["ss"] < 1e-4 and d["ds_mat"] < 1e-4 and d["k_prob"] < 1e-4, d
    assert d["perm_equal"], d
    net = fpm.Net(regression=True, backbone=False, dtype="bf16")
    net.load_state_dict(sd)
    with pytest.raises(AssertionError, match="UNIV_SIZE"):
        net.run(DeviceBatch.from_pairs(synth.make_batch(33, 1, [601], [64]), DEV))


# ---------------------------------------------------------------------------------------- probe x gallery (C4)
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_probe_gallery_shared_equals_per_pair(sd, dtype):
    """Computing the shared probe's SplineConv once and broadcasting it gives the per-pair results
    bit for bit (the per-graph stage does not depend on the partner)."""
    probe = synth.make_graph(40, 0, 0, 48)
    gallery = [synth.make_graph(40, p, 1, n) for p, n in enumerate([48, 40, 45, 48, 37, 48])]
    net = fpm.Net(regression=True, backbone=False, dtype=dtype)
    net.load_state_dict(sd)
    shared = DeviceBatch.from_probe_gallery(probe, gallery, DEV)
    plain = DeviceBatch.from_pairs([(probe, g) for g in gallery], DEV)
    a = net.run(shared, chunks=2)
    b = net.run(plain, chunks=2)
    for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert torch.equal(a[k], b[k]), k


def test_gemm_big_affinity_epilogue():
    """Vertex-affinity epilogue on the 256-row kernel (batched Kp^T: rows = graph-2 nodes)."""
    g = torch.Generator().manual_seed(9)
    B, M, N, K = 4, 256, 256, 768
    A = (torch.randn(B, M, K, generator=g) * 0.05).to(torch.bfloat16)
    Bm = (torch.randn(B, N, K, generator=g) * 0.05).to(torch.bfloat16)
    n1 = torch.tensor([256, 200, 131, 256], dtype=torch.int32)
    n2 = torch.tensor([256, 256, 99, 180], dtype=torch.int32)
    out = torch.empty(B, M, N, device=DEV)
    ops.gemm(A.to(DEV), Bm.to(DEV), M, N, K, K, K, batch=B, sA=M * K, sB=N * K, sC=M * N, epi=ops.EPI_AFFINITY,
             out_f=out, n1=n1.to(DEV), n2=n2.to(DEV))
    ref = torch.nn.functional.softplus(A.float() @ Bm.float().transpose(1, 2)) - 0.5
    for b in range(B):
        r, c = int(n2[b]), int(n1[b])
        assert (out[b, :r, :c].cpu() - ref[b, :r, :c]).abs().max() < 1e-4
        assert out[b, r:].abs().max().item() == 0 if r < M else True
        assert out[b, :, c:].abs().max().item() == 0 if c < N else True


def test_match_cls_bf16_vs_f32(sd):
    """bf16 conv2 (tap-major K on v_mfma_f32_16x16x16_bf16) against the fp32 path and the oracle's
    MatchClassifier: reported mode, logits within 2e-2 of the fp32 values (|logit| ~ 0.1-1)."""
    net = fpm.Net(regression=True, backbone=False, dtype="f32")
    net.load_state_dict(sd)
    wp = net.packed(DEV)
    g = torch.Generator().manual_seed(5)
    for B, n1, n2 in ((4, 256, 256), (3, 37, 50)):
        s = torch.randn(B, n1, n2, generator=g)
        perm = (torch.rand(B, n1, n2, generator=g) < 0.02).float()
        args = [wp[k] for k in ("mc_w1", "mc_b1", "mc_sc1", "mc_sh1", "mc_w2", "mc_b2", "mc_sc2", "mc_sh2", "mc_fcw",
                                "mc_fcb")]
        l32, _ = ops.match_cls(s.to(DEV), perm.to(DEV), *args, dtype=ops.F32)
        l16, _ = ops.match_cls(s.to(DEV), perm.to(DEV), *args, dtype=ops.BF16)
        ref = O.match_classifier(s * perm, sd)
        assert (l32.cpu() - ref).abs().max() < 1e-4
        assert (l16.cpu() - ref).abs().max() < 2e-2


def test_gnn_kernel_variants_bit_identical(sd):
    """Launch variants give bit-identical forwards: combine workgroup sizes, the global plan kernels,
    and the product GEMM on the 256 x 256 two-stage kernel (gemm_phase 0) instead of the phase
    kernel.  n = 96: above the fp64 k chain's 64-keypoint boxes, so the fp32 GNN layers and
    Sinkhorns run."""
    pairs = synth.make_batch(17, 3, 96)
    net = fpm.Net(regression=True, backbone=False, dtype="bf16")
    net.load_state_dict(sd)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    outs = []
    for key, val in (("combine_npb", 4), ("combine_npb", 16),
                     ("plan_graph", 0), ("gemm_phase", 0)):
        prev = ops.set_tuning(key, val)
        try:
            r = net.run(bt, chunks=1)
            torch.cuda.synchronize()
        finally:
            ops.set_tuning(key, prev)
        outs.append(r)
    for r in outs[1:]:
        for k in ("s", "ss", "ds_mat", "k_prob"):
            assert torch.equal(r[k], outs[0][k]), k


@pytest.mark.parametrize("P,nb", [(256, 5), (128, 5), (128, 4)])
def test_afau_gemm_norm_max_fused(P, nb):
    """AFA-U block tail fused into the FFN's second GEMM (fpm_gemm_norm_max): equal to the GEMM +
    separate instance norm + max (same GEMM accumulators; only the norm's reduction order differs)
    and to a float64 torch statement of InstanceNorm1d + max over positions.  P = 128: two pairs
    per 256-row tile (an odd pair count leaves the last tile half empty)."""
    g = torch.Generator().manual_seed(3)
    E, FF = 600, 256
    rows = nb * P
    A = torch.randn(rows, FF, generator=g).to(torch.bfloat16).to(DEV)
    W = (torch.randn(E, FF, generator=g) * 0.06).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(E, generator=g) * 0.1).to(DEV)
    res = torch.randn(rows, E, generator=g).to(DEV)
    nw = (torch.rand(E, generator=g) + 0.5).to(DEV)
    nbv = (torch.randn(E, generator=g) * 0.1).to(DEV)
    gm = ops.gemm_norm_max(A, W, rows, E, FF, FF, FF, bias, res, nw, nbv, torch.empty(nb, E, device=DEV), P=P)
    ff = torch.empty(rows, E, device=DEV)
    ops.gemm(A, W, rows, E, FF, FF, FF, bias=bias, out_f=ff, ldc=E)
    gm2 = torch.empty(nb, E, device=DEV)
    ops.instnorm(res, nb, P, E, nw, nbv, in2=ff, gmax=gm2)
    assert (gm - gm2).abs().max() < 2e-5
    v = (res.double() + (A.double() @ W.double().t() + bias.double())).view(nb, P, E)
    y = (v - v.mean(1, keepdim=True)) / torch.sqrt(v.var(1, unbiased=False, keepdim=True) + 1e-5)
    ref = (y * nw.double() + nbv.double()).max(1).values
    assert (gm.double() - ref).abs().max() < 1e-4
    with pytest.raises(fpm._lib.FpmError):
        ops.gemm_norm_max(A[:100], W, 100, E, FF, FF, FF, bias, res[:100], nw, nbv, gm, P=P)


@pytest.mark.parametrize("P,nb", [(256, 3), (128, 3)])
def test_afau_gemm_norm_out_fused(P, nb):
    """AFA-U block head fused into the attention-combine GEMM (fpm_gemm_norm_out): fp32 rows and the
    zero-K-padded bf16 copy equal to the GEMM + separate instance norm within reduction-order
    rounding, and to a float64 statement of InstanceNorm1d."""
    g = torch.Generator().manual_seed(4)
    E, K, KE = 600, 512, 640
    rows = nb * P
    A = torch.randn(rows, K, generator=g).to(torch.bfloat16).to(DEV)
    W = (torch.randn(E, K, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(E, generator=g) * 0.1).to(DEV)
    nw = (torch.rand(E, generator=g) + 0.5).to(DEV)
    nbv = (torch.randn(E, generator=g) * 0.1).to(DEV)
    o1f = torch.empty(rows, E, device=DEV)
    o1t = torch.full((rows, KE), 7.0, device=DEV).to(torch.bfloat16)
    ops.gemm_norm_out(A, W, rows, E, K, K, K, bias, nw, nbv, o1f, out_t=o1t, P=P)
    mh = torch.empty(rows, E, device=DEV)
    ops.gemm(A, W, rows, E, K, K, K, bias=bias, out_f=mh, ldc=E)
    r_f = torch.empty(rows, E, device=DEV)
    r_t = torch.empty(rows, KE, device=DEV).to(torch.bfloat16)
    ops.instnorm(mh, nb, P, E, nw, nbv, out_f=r_f, out_t=r_t, ldt=KE)
    assert (o1f - r_f).abs().max() < 2e-5
    assert (o1t.float() - r_t.float()).abs().max() <= 2 ** -6 * (r_f.abs().max() + 1)   # one bf16 ulp
    assert (o1t[:, E:] == 0).all()
    v = (A.double() @ W.double().t() + bias.double()).view(nb, P, E)
    y = (v - v.mean(1, keepdim=True)) / torch.sqrt(v.var(1, unbiased=False, keepdim=True) + 1e-5)
    ref = (y * nw.double() + nbv.double()).view(rows, E)
    assert (o1f.double() - ref).abs().max() < 1e-4


@pytest.mark.parametrize("afau,tol,n,B", [("bf16s", 2e-4, 256, 4), ("bf16x3", 1e-5, 256, 4), ("bf16x3", 1e-5, 128, 5)])
def test_afau_fused_forward_matches_unfused(sd, afau, tol, n, B):
    """Whole bf16 forwards with the fused AFA-U block head and tail agree with the unfused path on
    a 256-keypoint batch: ss identical (computed before AFA-U); k_prob within ``tol`` -- the fused
    first norm sums in another order, which can move a bf16 rounding of its operand copy by one
    ulp (bf16s: plain bf16 FFN operands, its k_prob distance from the fp32 oracle is ~4-8e-4;
    bf16x3: split near-fp32 operands written by the GEMM epilogues, fpm_gemm_x3out); the fp32 mode
    is not fused.  n = 128: two pairs per fused 256-row tile (five pairs: the last tile half empty)."""
    pairs = synth.make_batch(41, B, n)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    res = {}
    for fuse in (False, True):
        net = fpm.Net(regression=True, backbone=False, dtype="bf16", chunks=1, afau=afau)
        net.load_state_dict(sd)
        net.afau_fuse_norm = fuse
        res[fuse] = net.run(bt)
    assert (res[True]["k_prob"] - res[False]["k_prob"]).abs().max() < tol
    assert torch.equal(res[True]["ss"], res[False]["ss"])


def test_global_weights_kernel():
    """normalize_over_channels(cat(w1, w2)) (ngm.py:65-67, 262-268): within 1e-6 of the oracle, and a
    pair's row does not depend on how many pairs share the launch (shards / chunks computed alone)."""
    g = torch.Generator().manual_seed(31)
    w1, w2 = torch.rand(7, 512, generator=g), torch.rand(7, 512, generator=g) * 3
    full = ops.global_weights(w1.to(DEV), w2.to(DEV))
    assert (full.cpu() - O.global_weights(w1, w2)).abs().max() < 1e-6
    part = ops.global_weights(w1[2:5].to(DEV), w2[2:5].to(DEV))
    assert torch.equal(part, full[2:5])


def test_split_bf16x3_operands():
    """[hi | lo | hi] split rows: hi = bf16(x), hi + lo within 2^-16 of x, zero K padding; packed
    [W_hi | W_hi | W_lo] weights give a product within 1e-5 (relative) of the fp32 one."""
    g = torch.Generator().manual_seed(32)
    x = torch.randn(37, 600, generator=g)
    s3 = ops.split_bf16x3(x.to(DEV), 640).cpu()
    hi, lo, hi2 = s3[:, :640].float(), s3[:, 640:1280].float(), s3[:, 1280:].float()
    assert torch.equal(hi[:, :600], x.to(torch.bfloat16).float()) and torch.equal(hi, hi2)
    assert (hi[:, 600:] == 0).all() and (lo[:, 600:] == 0).all()
    assert ((hi + lo)[:, :600] - x).abs().max() <= x.abs().max() * 2.0 ** -16
    W = torch.randn(256, 600, generator=g) * 0.05
    W3 = ops.split_weights_bf16x3(W.to(DEV), 640)
    out = torch.empty(37, 256, device=DEV)
    ops.gemm(s3.to(DEV), W3, 37, 256, 1920, 1920, 1920, out_f=out)
    ref = x.double() @ W.double().t()
    assert ((out.cpu().double() - ref).abs().max() / ref.abs().max()) < 1e-5


def test_crossset_attn_split_rows(sd):
    """The attention kernel's split store (dtype 2): hi equals the bf16 store bit for bit (same
    arithmetic), hi + lo is the unrounded value (within 2^-16)."""
    net = fpm.Net(regression=True, dtype="bf16", backbone=False)
    net.load_state_dict(sd)
    wp = net.packed(DEV)
    g = torch.Generator().manual_seed(33)
    B, n = 3, 64
    ss = (torch.rand(B, n, n, generator=g) ** 4).to(DEV)
    n2 = _i32([64, 50, 61])
    args = [wp[k] for k in ("row_Wv", "row_mix1w", "row_mix1b", "row_mix2w", "row_mix2b")]
    a16 = torch.empty(B * n, 256, device=DEV, dtype=torch.bfloat16)
    ops.crossset_attn(ss, n2, *args, a16)
    a3 = torch.empty(B * n, 768, device=DEV, dtype=torch.bfloat16)
    ops.crossset_attn(ss, n2, *args, a3, split=True)
    assert torch.equal(a3[:, :256], a16) and torch.equal(a3[:, 512:], a16)
    full = a3[:, :256].float() + a3[:, 256:512].float()
    assert (full - a16.float()).abs().max() <= full.abs().max() * 2.0 ** -8


@pytest.mark.parametrize("n,n2", [(256, [256, 256]), (40, [40, 31, 26]), (512, [512])])
def test_plan_per_graph_equals_global(n, n2):
    """The per-graph spline plan (one workgroup per graph, LDS sort) and the global plan give the
    same CSR, product rows and GEMM tile tables: SplineConv outputs and the GNN CSR bit-identical."""
    pairs = synth.make_batch(50 + n, len(n2), n, n2=n2)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    for side in range(2):
        nn_ = bt.B * bt.nmax[side]
        me = bt.max_graph_edges(side)
        assert me > 0
        p1 = ops.spline_plan(bt.src[side], bt.dst[side], bt.pseudo[side], nn_, bt.nmax[side], me)
        p0 = ops.spline_plan(bt.src[side], bt.dst[side], bt.pseudo[side], nn_, bt.nmax[side], 0)
        E = bt.E[side]
        c1, c0 = ops.plan_csr(p1, E, nn_), ops.plan_csr(p0, E, nn_)
        base1, base0 = p1.data_ptr(), p0.data_ptr()
        ptr1 = p1[c1[0] - base1:c1[0] - base1 + 4 * (nn_ + 1)].view(torch.int32)
        ptr0 = p0[c0[0] - base0:c0[0] - base0 + 4 * (nn_ + 1)].view(torch.int32)
        nb1 = p1[c1[1] - base1:c1[1] - base1 + 4 * E].view(torch.int32)
        nb0 = p0[c0[1] - base0:c0[1] - base0 + 4 * E].view(torch.int32)
        assert torch.equal(ptr1, ptr0) and torch.equal(nb1, nb0)
        a1, o1 = ops.spline_plan_rows(p1, E, nn_)
        a0, o0 = ops.spline_plan_rows(p0, E, nn_)
        assert torch.equal(o1, o0)
        tot = int(o0[26].item())
        assert torch.equal(a1[:tot], a0[:tot])
    net = fpm.Net(regression=True, dtype="f32", backbone=False)
    outs = []
    for v in (1, 0):
        prev = ops.set_tuning("plan_graph", v)
        try:
            outs.append(net.run_gpu_stage(bt, keep_feats=True))
            torch.cuda.synchronize()
        finally:
            ops.set_tuning("plan_graph", prev)
    for k in ("feat0", "feat1", "s", "ss"):
        assert torch.equal(outs[0][k], outs[1][k]), k


# ------------------------------------------------------------------------------------- bf16 cast
@pytest.mark.parametrize("n", [768 * 300, 8 * 7, 13, 1000003])
def test_cast_bf16_round_to_nearest_even(n):
    """fpm_cast_bf16 (16-B vector path when n % 8 == 0, scalar tail path otherwise) equals torch's
    round-to-nearest-even float32 -> bfloat16 conversion bit for bit."""
    g = torch.Generator().manual_seed(n)
    x = (torch.randn(n, generator=g) * torch.exp(torch.randn(n, generator=g) * 4)).to(DEV)
    y = ops.cast_bf16(x)
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int16), x.to(torch.bfloat16).view(torch.int16))


@pytest.mark.parametrize("B,n1,n2max,n2s", [(5, 256, 256, [256, 250, 256, 241, 256]), (2, 100, 512, [512, 437])])
def test_crossset_attn_head_split_bitwise(sd, B, n1, n2max, n2s):
    """The LDS-V attention kernel with its 16 heads split over 1 / 2 / 4 / 8 / 16 workgroups per row
    block (small launches) writes the same outputs and softmax stats bit for bit, in every mode."""
    net = fpm.Net(regression=True, dtype="bf16", backbone=False)
    net.load_state_dict(sd)
    wp = net.packed(DEV)
    g = torch.Generator().manual_seed(n1 + 7)
    ss = (torch.rand(B, n1, n2max, generator=g) ** 4).to(DEV)
    n2 = _i32(n2s)
    args = [wp[k] for k in ("row_Wv", "row_mix1w", "row_mix1b", "row_mix2w", "row_mix2b")]
    res = {}
    for z in (1, 2, 4, 8, 16):
        pz = ops.set_tuning("afau_head_split", z)
        try:
            o32 = torch.empty(B * n1, 256, device=DEV)
            st = torch.empty(B * n1, 16, 2, device=DEV)
            ops.crossset_attn(ss, n2, *args, o32, stats=st)
            o3 = torch.empty(B * n1, 768, device=DEV, dtype=torch.bfloat16)
            ops.crossset_attn(ss, n2, *args, o3, split=True)
            torch.cuda.synchronize()
        finally:
            ops.set_tuning("afau_head_split", pz)
        res[z] = (o32, st, o3)
    for z in (2, 4, 8, 16):
        for a, b in zip(res[1], res[z]):
            assert torch.equal(a, b), z


@pytest.mark.parametrize("B,n1,n2max,n2s", [(3, 64, 64, [64, 50, 61]), (2, 200, 256, [256, 233]), (2, 37, 45, [45, 20]),
                                             (2, 100, 512, [512, 437]), (1, 40, 301, [301])])
def test_crossset_attn_lds_v_kernel(sd, B, n1, n2max, n2s):
    """The LDS-staged-V attention kernel (n2max <= 256) against the global-V kernel with the same
    16-term scores: fp32 outputs and softmax stats within fp32 summation-order rounding; the bf16
    mode's interval-classified scores (exact up to reassociation) against the fp32 kernel."""
    net = fpm.Net(regression=True, dtype="bf16", backbone=False)
    net.load_state_dict(sd)
    wp = net.packed(DEV)
    g = torch.Generator().manual_seed(n1 + n2max)
    ss = (torch.rand(B, n1, n2max, generator=g) ** 4).to(DEV)
    n2 = _i32(n2s)
    args = [wp[k] for k in ("row_Wv", "row_mix1w", "row_mix1b", "row_mix2w", "row_mix2b")]
    res = {}
    for v in (0, 1):
        pv = ops.set_tuning("afau_attn_v", v)
        try:
            o32 = torch.empty(B * n1, 256, device=DEV)
            st = torch.empty(B * n1, 16, 2, device=DEV)
            ops.crossset_attn(ss, n2, *args, o32, stats=st)
            o3 = torch.empty(B * n1, 768, device=DEV, dtype=torch.bfloat16)
            ops.crossset_attn(ss, n2, *args, o3, split=True)
            torch.cuda.synchronize()
        finally:
            ops.set_tuning("afau_attn_v", pv)
        res[v] = (o32, st, o3[:, :256].float() + o3[:, 256:512].float())
    (a0, s0, _), (a1, s1, h1) = res[0], res[1]
    scale = a0.abs().max()
    assert (a1 - a0).abs().max() <= 1e-5 * scale
    assert torch.allclose(s1, s0, rtol=1e-5, atol=1e-6)
    assert (h1 - a0).abs().max() <= 2e-5 * scale




# ------------------------------------------------ ngm.py pieces pinned by the reference's own source
def test_device_tail_vs_reference_fixture():
    """The device AFA-U k head, soft top-k, selection and MatchClassifier on the inputs of the
    reference-executed ngm.py:373-487 fixture (tests/golden/ngm_tail.npz, make_golden.py): k_prob,
    ds_mat and cls_prob within 1e-4 of the REFERENCE's outputs, perm_mat identical; and the
    node-classifier readout (ngm.py:368-369) against its fixture; perm_mat identical or explained pair
    by pair (a pick among matches tied in the reference's ds_mat)."""
    import types
    z = np.load(os.path.join(GOLDEN, "ngm_tail.npz"))
    sd = params.init_params(int(z["seed"]))
    net = fpm.Net(regression=True, backbone=False)
    net.load_state_dict(sd)
    wp = net.packed(DEV)
    for c in range(int(z["ncases"])):
        g = lambda k: torch.from_numpy(np.asarray(z["c%d_%s" % (c, k)]))
        s, ss = g("s").to(DEV).contiguous(), g("ss").to(DEV).contiguous()
        B, n1max, n2max = s.shape
        n1h, n2h = g("n1").to(torch.int32), g("n2").to(torch.int32)
        bt = types.SimpleNamespace(B=B, n1max=n1max, n2max=n2max, n1=n1h.to(DEV), n2=n2h.to(DEV),
                                   n_host=(n1h, n2h), device=DEV)
        ks = net._afau(wp, ss, bt)
        min_pt = torch.minimum(bt.n1, bt.n2).float()
        kk = (ks * min_pt).contiguous()
        steps = torch.empty(B, device=DEV, dtype=torch.int32)
        ds = ops.soft_topk_fwd(ss, bt.n1, bt.n2, kk, 10, 0.01, steps=steps)
        assign = ops.lsa_batch_host(ds.cpu(), n1h, n2h, 2)
        perm = ops.topk_select(ds, assign.to(DEV), kk)
        logits, prob = ops.match_cls(s, perm.contiguous(), wp["mc_w1"], wp["mc_b1"], wp["mc_sc1"], wp["mc_sh1"],
                                     wp["mc_w2"], wp["mc_b2"], wp["mc_sc2"], wp["mc_sh2"], wp["mc_fcw"], wp["mc_fcb"])
        d = {"k_prob": float((ks.cpu() - g("ks")).abs().max()), "ds_mat": float((ds.cpu() - g("ds_mat")).abs().max()),
             "cls_logits": float((logits.cpu() - g("cls_logits")).abs().max()),
             "cls_prob": float((prob.cpu() - g("cls_prob")).abs().max())}
        print("case", c, d)
        assert d["k_prob"] < 1e-4 and d["ds_mat"] < 1e-4 and d["cls_prob"] < 1e-4, (c, d)
        # perm_mat: identical, or a different pick among matches the reference's own ds_mat ties within
        # 1e-5 (soft top-k saturates at 1.0; oracle.compare), or a k* rounding crossing
        for b in range(B):
            m = int(min(n1h[b], n2h[b]))
            cls = O.compare.classify_pair(perm[b].cpu(), g("perm")[b], g("ds_mat")[b], k=ks[b].cpu(),
                                          k_ref=g("ks")[b], m=m, k_tol=1e-4)
            assert cls != "mismatch", (c, b, cls)
    B, n1max, n2max = 2, int(z["readout_n1max"]), int(z["readout_n2max"])
    emb = torch.from_numpy(z["readout_emb"])
    X = emb.view(B, n2max, n1max, 17).permute(0, 3, 1, 2).contiguous().to(DEV)
    s = torch.empty(B, n1max, n2max, device=DEV)
    ops.node_classifier(X, B, n1max, n2max, wp["cls_w"], wp["cls_b"], s)
    assert float((s.cpu() - torch.from_numpy(z["readout_s"])).abs().max()) < 1e-5


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_device_match_classifier_vs_reference_fixture(dtype):
    """MatchClassifier (ngm.py:75-106) in eval mode, reference-executed on the fixture's matrices
    (tests/golden/match_classifier.npz): the HIP classifier's logits within 2e-5 (fp32 path) /
    2e-2 on the bf16 conv2 path (as test_match_cls_bf16_vs_f32)."""
    z = np.load(os.path.join(GOLDEN, "match_classifier.npz"))
    sd = params.init_params(int(z["seed"]))
    net = fpm.Net(regression=True, backbone=False)
    net.load_state_dict(sd)
    wp = net.packed(DEV)
    m = torch.from_numpy(z["m"]).to(DEV)
    # the kernel takes s and perm separately (conv1 fuses s * perm): perm = 1 where the fixture is set
    perm = (m != 0).float()
    logits, _ = ops.match_cls(m.contiguous(), perm, wp["mc_w1"], wp["mc_b1"], wp["mc_sc1"], wp["mc_sh1"],
                              wp["mc_w2"], wp["mc_b2"], wp["mc_sc2"], wp["mc_sh2"], wp["mc_fcw"], wp["mc_fcb"],
                              dtype=ops.BF16 if dtype == "bf16" else ops.F32)
    err = float((logits.cpu() - torch.from_numpy(z["logits_eval"])).abs().max())
    print(dtype, "max |d logits|", err)
    assert err < (2e-5 if dtype == "f32" else 2e-2), err


# ------------------------------------------- gate-passing fast mode: bf16 SplineConv + bf16x3 AFA-U
@pytest.mark.parametrize("epi", ["store", "relu", "norm_out"])
def test_gemm_x3out_epilogues(epi):
    """fpm_gemm_x3out: the fp32 result on the 256-row bf16 MFMA tile written straight as split
    [hi | lo | hi] operands -- bit-identical to fpm_split_bf16x3 of its own fp32 rows, zero K padding
    in every segment, fp32 rows equal to the plain fp32-output GEMM (same accumulators) or, for the
    norm epilogue, to fpm_gemm_norm_out bit for bit."""
    g = torch.Generator().manual_seed(7)
    nb, P = 3, 256
    rows = nb * P
    N, K, Kp = (600, 768, 640) if epi != "relu" else (256, 1920, 256)
    A = torch.randn(rows, K, generator=g).to(torch.bfloat16).to(DEV)
    W = (torch.randn(N, K, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    bias = (torch.randn(N, generator=g) * 0.1).to(DEV)
    nw = (torch.rand(N, generator=g) + 0.5).to(DEV)
    nbv = (torch.randn(N, generator=g) * 0.1).to(DEV)
    code = {"store": ops.EPI_STORE, "relu": ops.EPI_RELU, "norm_out": ops.EPI_NORM_OUT}[epi]
    out_f = torch.empty(rows, N, device=DEV)
    o3 = torch.full((rows, 3 * Kp), 3.0, device=DEV).to(torch.bfloat16)
    ops.gemm_x3out(A, W, rows, N, K, Kp, epi=code, bias=bias, out_t3=o3, out_f=out_f, nw=nw, nb=nbv)
    assert torch.equal(o3, ops.split_bf16x3(out_f, Kp))
    ref = torch.empty(rows, N, device=DEV)
    if epi == "norm_out":
        ops.gemm_norm_out(A, W, rows, N, K, K, K, bias, nw, nbv, ref)
    else:
        ops.gemm(A, W, rows, N, K, K, K, epi=code, bias=bias, out_f=ref, ldc=N)
    assert torch.equal(out_f, ref)
    # without the fp32 rows: the same split rows
    o3b = ops.gemm_x3out(A, W, rows, N, K, Kp, epi=code, bias=bias, out_f=out_f if epi == "norm_out" else None,
                         nw=nw, nb=nbv)
    assert torch.equal(o3b, o3)
    with pytest.raises(fpm._lib.FpmError):
        ops.gemm_x3out(A, W, rows, N, K, N - 4, epi=code, bias=bias)          # segment shorter than N


GATE = {"ss": 1e-4, "ds_mat": 1e-4, "k_prob": 1e-4}   # north star: soft permutation + predicted k, 1e-4 fp32


def _gated(pairs, sd, name, bt=None):
    """The gate-passing fast mode (dtype bf16, AFA-U bf16x3) against the fp32 oracle: ss / ds_mat /
    k_prob within 1e-4 (GATE), per-stage deltas recorded (Kp, s, cls_prob), perm_mat identical or
    explained pair by pair (oracle.compare with the 1e-4 k tolerance)."""
    net = fpm.Net(regression=True, backbone=False, dtype="bf16", afau="bf16x3")
    net.load_state_dict(sd)
    res = net.run(bt if bt is not None else DeviceBatch.from_pairs(pairs, DEV))
    ref = O.forward(pairs, sd, regression=True)
    d = {k: float((res[k].float().cpu() - ref[k]).abs().max()) for k in ("Kp", "s", "ss", "ds_mat", "k_prob", "cls_prob")}
    rep = O.compare.perm_report(res, ref, [p[0]["n"] for p in pairs], [p[1]["n"] for p in pairs],
                                reduced_precision=True, k_tol=GATE["k_prob"])
    d["perm_classes"] = rep["counts"]
    _record(name, d)
    for k, tol in GATE.items():
        assert d[k] < tol, (k, d)
    assert rep["counts"]["mismatch"] == 0, rep
    return d


def test_gated_mode_c2(sd):
    """C2's graph size (n = 128, 6 pairs; the unfused bf16x3 AFA-U path: P != 256)."""
    _gated(synth.make_batch(13, 6, 128), sd, "gated_c2")


def test_gated_mode_c3(sd):
    """C3 (n = 256, 16 pairs; the fused bf16x3 AFA-U path)."""
    _gated(synth.make_batch(5, 16, 256), sd, "gated_c3")


def test_gated_mode_c3_ragged(sd):
    """C3-sized ragged batch (n1max = 256 fused path with padded pairs, transposed Sinkhorn)."""
    _gated(synth.make_batch(71, 4, [256, 240, 251, 230], n2=[247, 256, 233, 256]), sd, "gated_c3_ragged")


def test_gated_mode_c4(sd):
    """C4 (1 probe x gallery, n = 128, probe SplineConv shared)."""
    probe = synth.make_graph(17, 0, 0, 128)
    gallery = [synth.make_graph(17, 1 + g, 1, 128 - (g % 3) * 5) for g in range(6)]
    pairs = [(probe, g) for g in gallery]
    _gated(pairs, sd, "gated_c4", bt=DeviceBatch.from_probe_gallery(probe, gallery, DEV))


@pytest.mark.slow
def test_gated_mode_c5(sd):
    """C5 (n = 512, streaming Sinkhorn / soft top-k, unfused AFA-U)."""
    _gated(synth.make_batch(62, 2, 512), sd, "gated_c5")


def test_affinity_fwd_vs_reference_golden():
    """fpm_affinity_fwd (the surveyed C-ABI entry) against the reference's own
    InnerProductWithWeightsAffinity output (tests/golden/affinity.npz, ragged pairs 7 x 9 and
    5 x 5): within 1e-5, zero outside each pair's block; the edge form is half of softplus - 0.5."""
    z = np.load(os.path.join(GOLDEN, "affinity.npz"))
    sd_ = params.init_params(int(z["seed"]))
    X = [torch.from_numpy(z["X%d" % i]) for i in range(2)]
    Y = [torch.from_numpy(z["Y%d" % i]) for i in range(2)]
    n1 = torch.tensor([x.shape[0] for x in X], dtype=torch.int32)
    n2 = torch.tensor([y.shape[0] for y in Y], dtype=torch.int32)
    X1 = torch.zeros(2, int(n1.max()), 768)
    X2 = torch.zeros(2, int(n2.max()), 768)
    for b in range(2):
        X1[b, :n1[b]] = X[b]
        X2[b, :n2[b]] = Y[b]
    args = [t.to(DEV) for t in (X1, X2, torch.from_numpy(z["W"]), sd_["vertex_affinity.A.weight"],
                                sd_["vertex_affinity.A.bias"], n1, n2)]
    K = ops.affinity(*args).cpu()
    for b in range(2):
        ref = torch.from_numpy(z["K%d" % b])
        assert (K[b, :n1[b], :n2[b]] - ref).abs().max() < 1e-5, b
        assert K[b, n1[b]:].abs().max() == 0 if n1[b] < K.shape[1] else True
        assert K[b, :, n2[b]:].abs().max() == 0 if n2[b] < K.shape[2] else True
    Kh = ops.affinity(*args, half=True).cpu()
    assert (Kh - 0.5 * K).abs().max() < 1e-6


def test_one_chunk_tail_groups_bitwise(sd):
    """A one-chunk forward whose tail (AFA-U, soft top-k, ds_mat D2H) runs in pair groups, each
    group's host Hungarian starting while the GPU works on the next, on one stream or rotating
    over two or three: every output equal bit for bit to the ungrouped tail (per-pair kernels; the
    AFA-U column block is shared by offset)."""
    pairs = synth.make_batch(47, 50, 32, n2=[32 - (b % 4) for b in range(50)])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    res = {}
    for groups, streams in ((1, 1), (3, 1), (3, 2), (3, 3)):
        net = fpm.Net(regression=True, backbone=False, dtype="bf16", chunks=1)
        net.load_state_dict(sd)
        net.tail_groups, net.tail_streams = groups, streams
        res[groups, streams] = {k: v.clone() for k, v in net.run(bt).items() if torch.is_tensor(v)}
        assert net.last_timing["host_units"] == groups
    for k in ("s", "ss", "ds_mat", "perm_mat", "lsa", "k_prob", "cls_prob", "sk_steps"):
        assert torch.equal(res[1, 1][k], res[3, 1][k]), k
        assert torch.equal(res[1, 1][k], res[3, 2][k]), k     # groups alternating over two streams
        assert torch.equal(res[1, 1][k], res[3, 3][k]), k     # three groups, one stream each


@pytest.mark.parametrize("B,chunks", [(50, 1), (300, None)])
def test_zero_copy_ds_mat_bitwise(sd, B, chunks):
    """ds_mat for the host Hungarian written to pinned memory by the soft top-k kernel itself
    (zero-copy, Net.zero_copy 1 / 2) instead of the copy stream's D2H: every output identical bit for
    bit -- one-chunk forwards with tail groups and multi-chunk pipelines."""
    pairs = synth.make_batch(53, B, 32, n2=[32 - (b % 4) for b in range(B)])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    res = {}
    for zc in (0, 1, 2):
        net = fpm.Net(regression=True, backbone=False, dtype="bf16", chunks=chunks)
        net.load_state_dict(sd)
        net.zero_copy = zc
        if chunks is None:
            net.pipeline_chunks = lambda B_: 4
        res[zc] = net.run(bt)
    for zc in (1, 2):
        for k in ("s", "ss", "ds_mat", "perm_mat", "lsa", "k_prob", "cls_prob", "sk_steps"):
            assert torch.equal(res[0][k], res[zc][k]), (zc, k)


def test_batch_vs_solo_bitwise(sd):
    """A pair's outputs do not depend on the batch around it (the bench's timed-batch self-check,
    at test size): a 140-pair n = 256 bf16 batch (large enough that the affinity GEMM takes the
    256-row kernels) against each checked pair re-run alone with the same padded box, which takes
    the small-tile GEMM -- the two kernels' affinity epilogues must agree bit for bit."""
    pairs = synth.make_batch(49, 140, 256, n2=[256 - (b % 7) for b in range(140)])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    net = fpm.Net(regression=True, backbone=False, dtype="bf16")
    net.load_state_dict(sd)
    res = net.run(bt)
    for b in (0, 77, 139):
        solo = net.run(bt.split_range(b, b + 1), chunks=1)
        for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob"):
            assert torch.equal(solo[k][0], res[k][b]), (b, k)


def test_gnn_channel_sweeps_bit_identical(sd):
    """The GNN layer's phase-1 channel-group sweeps (gnn_sweeps = 2, 3: one pass over the neighbour
    rows per channel group) keep every channel's neighbour-list order: outputs equal the one-pass
    kernel's bit for bit."""
    pairs = synth.make_batch(50, 6, 64, n2=[64, 61, 64, 58, 64, 64])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    res = {}
    for v in (1, 2, 3):
        prev = ops.set_tuning("gnn_sweeps", v)
        try:
            net = fpm.Net(regression=True, backbone=False, dtype="bf16")
            net.load_state_dict(sd)
            res[v] = net.run(bt)
        finally:
            ops.set_tuning("gnn_sweeps", prev)
    for v in (2, 3):
        for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob"):
            assert torch.equal(res[1][k], res[v][k]), (v, k)


def test_store_cache_policies_bit_identical(sd):
    """The sc1 store variants (gnn_store_sc1, combine_store_sc1, gemm_store_sc1: the written lines
    leave the XCD's L2) change where bytes are cached, never the bytes: a bf16 and an fp32 forward
    with every switch off equal the default ones bit for bit."""
    pairs = synth.make_batch(48, 6, 64, n2=[64, 60, 64, 57, 64, 64])
    bt = DeviceBatch.from_pairs(pairs, DEV)
    keys = ("gnn_store_sc1", "combine_store_sc1", "gemm_store_sc1")
    for dtype in ("bf16", "f32"):
        res = {}
        for v in (1, 0):
            prev = [(k, ops.set_tuning(k, v)) for k in keys]
            try:
                net = fpm.Net(regression=True, backbone=False, dtype=dtype)
                net.load_state_dict(sd)
                res[v] = net.run(bt)
            finally:
                for k, pv in prev:
                    ops.set_tuning(k, pv)
        for k in ("s", "ss", "ds_mat", "perm_mat", "k_prob", "cls_prob"):
            assert torch.equal(res[0][k], res[1][k]), (dtype, k)
