"""Image front end: ResNet-18 backbone (fpm.backbone, MIOpen convolutions) +
the fused normalise / feature_align / concat / global-max-pool kernel (fpm_feature_align_fwd), and
the full images -> match forward through Net(backbone=True).

Oracle: oracle/frontend_oracle.py, pinned bit-exactly by tests/golden/feature_align.npz (the
reference's own utils/feature_align.py).  GPU tolerance: 2e-6 abs on the aligned features (the
channel norm's summation order differs from torch's; the interpolation itself is evaluated in the
reference's fp32 operation order without FMA contraction).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import frontend_oracle as FO


def _golden():
    z = np.load(os.path.join(GOLDEN, "feature_align.npz"))
    return {k: torch.from_numpy(z[k]) for k in z.files}


def test_oracle_feature_align_golden():
    z = _golden()
    U = FO.feature_align(FO.normalize_over_channels(z["nodes"]), z["P"], z["ns"])
    F = FO.feature_align(FO.normalize_over_channels(z["edges"]), z["P"], z["ns"])
    assert torch.equal(U, z["U"]) and torch.equal(F, z["F"])


def test_image_fixture_is_ill_conditioned():
    """The committed MIOpen-feature fixture (tests/golden/image_feats_miopen.npz, see
    test_image_fixture_k_vs_exact) is the kind of input the k gate is anchored for: the fp32
    reference's own k_prob sits > 5e-5 from its fp64 value on the unpadded pair, and its two valid
    fp32 evaluation orders (factorised vs the literal explicit-pattern SAGE mean) disagree there."""
    import oracle as O
    from fpm import params
    z = np.load(os.path.join(GOLDEN, "image_feats_miopen.npz"))
    pairs = _pairs_from_feats([z["x0"], z["x1"]], [z["g0"], z["g1"]], [z["P0"], z["P1"]], [z["n0"], z["n1"]])
    sd = params.init_params(5)
    k32 = O.forward(pairs, sd)["k_prob"].double()
    k32x = O.forward(pairs, sd, explicit_pattern=True)["k_prob"].double()
    k64 = O.forward(pairs, sd, dtype=torch.float64)["k_prob"]
    floor = torch.maximum((k32 - k64).abs(), (k32x - k64).abs())
    assert float(floor[0]) > 5e-5, floor
    assert float((k32 - k32x).abs().max()) > 1e-5


def test_backbone_layout_and_shapes():
    """torchvision resnet18 names inside the reference's Sequential split; stride-16 / stride-32
    maps of a 240x320 image are 15x20x256 and 8x10x512 (feature_extractor.py:46-58)."""
    from fpm.backbone import build_resnet18_split, backbone_state_dict
    sd = backbone_state_dict(0)
    for k, shape in (("node_layers.0.weight", (64, 3, 7, 7)), ("node_layers.1.running_var", (64,)),
                     ("node_layers.4.0.conv1.weight", (64, 64, 3, 3)),
                     ("node_layers.5.0.downsample.0.weight", (128, 64, 1, 1)),
                     ("node_layers.6.1.bn2.bias", (256,)), ("edge_layers.0.0.downsample.1.weight", (512,)),
                     ("edge_layers.0.1.conv2.weight", (512, 512, 3, 3))):
        assert tuple(sd[k].shape) == shape, k
    assert sum(v.numel() for k, v in sd.items() if not k.endswith("num_batches_tracked")) == 11176512 + 9600
    nl, el, fl = build_resnet18_split(0)
    nl.eval()
    el.eval()
    with torch.no_grad():
        nodes = nl(torch.randn(1, 3, 240, 320))
        edges = el(nodes)
    assert nodes.shape == (1, 256, 15, 20) and edges.shape == (1, 512, 8, 10)
    assert fl(edges).shape == (1, 512, 1, 1)


# ------------------------------------------------------------------------------- GPU
DEV = torch.device("cuda", 0)


@pytest.fixture
def deterministic_convs():
    """Ask the library convolutions for deterministic algorithms where they have them."""
    with torch.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=True):
        yield


@pytest.mark.gpu
@pytest.mark.parametrize("channels_last", [False, True])
def test_feature_align_kernel_golden(channels_last):
    from fpm import ops
    z = _golden()
    mf = torch.channels_last if channels_last else torch.contiguous_format
    nodes = z["nodes"].to(DEV).contiguous(memory_format=mf)
    edges = z["edges"].to(DEV).contiguous(memory_format=mf)
    B, nmax = z["P"].shape[:2]
    n = z["ns"].to(torch.int32).to(DEV)
    X, g = ops.feature_align(nodes, edges, z["P"].to(DEV), n)
    X = X.cpu().view(B, nmax, -1)
    U, F = z["U"].transpose(1, 2), z["F"].transpose(1, 2)
    cn = U.shape[-1]
    assert (X[..., :cn] - U).abs().max() < 2e-6
    assert (X[..., cn:] - F).abs().max() < 2e-6
    for b in range(B):
        assert not X[b, int(z["ns"][b]):].any()
    assert torch.equal(g.cpu(), torch.amax(z["edges"], dim=(2, 3)))


def _image_batch(B, n, seed):
    g = torch.Generator().manual_seed(seed)
    imgs = [torch.rand(B, 3, 240, 320, generator=g) for _ in range(2)]
    Ps, ns = [], []
    rng = np.random.default_rng(seed)
    for side in range(2):
        P = np.zeros((B, n, 2), np.float32)
        nn_ = []
        for b in range(B):
            m = n - (b % 3) * 5
            P[b, :m] = np.stack([rng.uniform(0, 320, m), rng.uniform(0, 240, m)], 1)
            nn_.append(m)
        Ps.append(torch.from_numpy(P))
        ns.append(torch.tensor(nn_))
    return imgs, Ps, ns


@pytest.mark.gpu
def test_image_features_vs_oracle():
    """Backbone on MIOpen + HIP align vs the same backbone on CPU + the oracle front end."""
    import fpm
    net = fpm.Net(regression=True, backbone=True)
    imgs, Ps, ns = _image_batch(2, 40, 3)
    xs, gs = net.image_features(imgs, Ps, ns, DEV)
    from fpm.backbone import build_resnet18_split
    nl, el, _ = build_resnet18_split(0)
    nl.eval()
    el.eval()
    for side in range(2):
        with torch.no_grad():
            nodes = nl(imgs[side])
            edges = el(nodes)
        xr, gr = FO.image_features(nodes, edges, Ps[side], ns[side])
        assert (xs[side].cpu().view_as(xr) - xr).abs().max() < 1e-4
        assert (gs[side].cpu() - gr).abs().max() < 1e-3 * max(1.0, float(gr.abs().max()))


def _dump_feats(name, xs, gs, Ps, ns):
    """The captured matcher inputs of a run, for a fixture (tests/golden/image_feats_*.npz)."""
    outd = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")
    os.makedirs(outd, exist_ok=True)
    np.savez_compressed(os.path.join(outd, name), x0=xs[0].cpu().numpy(), x1=xs[1].cpu().numpy(),
                        g0=gs[0].cpu().numpy(), g1=gs[1].cpu().numpy(), P0=Ps[0].numpy(), P1=Ps[1].numpy(),
                        n0=ns[0].numpy(), n1=ns[1].numpy())


def _pairs_from_feats(xs, gs, Ps, ns):
    from oracle import graphs_oracle as GO
    B, n = Ps[0].shape[:2]
    pairs = []
    for b in range(B):
        pr = []
        for side in range(2):
            m = int(ns[side][b])
            p = np.asarray(Ps[side][b, :m])
            A = GO.delaunay_triangulate(p.astype(np.float64))
            ei, attr = GO.pyg_edges(A, p)
            x = np.asarray(xs[side]).reshape(B, n, -1)[b, :m]
            pr.append(dict(n=m, x=x, w=np.asarray(gs[side][b]), edge_index=ei, pseudo=attr, P=p, A=A))
        pairs.append(tuple(pr))
    return pairs


@pytest.mark.gpu
def test_images_to_match_forward():
    """data_dict with only images / Ps / ns (+ gt, label): backbone, feature_align, device Delaunay
    graphs and the matcher, through Net.forward.  Device-built graphs give the same result bit for
    bit as host-built (scipy) ones; on the features this forward computed (captured: MIOpen's
    features vary run to run, the oracle sees the identical ones) ds_mat is within 1e-4 of the fp32
    oracle and k_prob passes the k gate (_k_gate: within 1e-4 beyond the fp32 reference's own
    deviation from the exact value, and -- the fp64 k chain runs on these 32-keypoint boxes --
    within 2e-5 of the exact value itself).  A failing run leaves its inputs in
    gpurun_out/images_to_match_feats.npz (FPM_DUMP_FEATS=1: every run)."""
    import fpm
    from fpm import params
    from fpm.batch import DeviceBatch
    import oracle as O
    net = fpm.Net(regression=True, backbone=True)
    sd = params.init_params(5)
    net.load_state_dict({**net.state_dict(), **sd})
    B, n = 3, 32
    imgs, Ps, ns = _image_batch(B, n, 8)
    dd = {"images": imgs, "Ps": Ps, "ns": ns, "gt_perm_mat": torch.zeros(B, n, n)}
    # the features this forward computed (MIOpen may pick a different convolution algorithm on
    # another call, so a second image_features call is not bit-identical)
    seen = {}
    image_features = net.image_features

    def spy(*a, **kw):
        seen["f"] = image_features(*a, **kw)
        return seen["f"]

    net.image_features = spy
    try:
        out = net.forward(dict(dd))
    finally:
        net.image_features = image_features
    xs, gs = seen["f"]
    xs_h = [x.view(B, n, -1).cpu().numpy() for x in xs]
    gs_h = [g.cpu().numpy() for g in gs]
    pairs = _pairs_from_feats(xs_h, gs_h, Ps, ns)
    ref = net.run(DeviceBatch.from_pairs(pairs, DEV), gt_perm=dd["gt_perm_mat"])
    # same features, graphs built on the device from Ps (no pyg_graphs): bit-identical
    dd2 = {"node_features": [x.view(B, n, -1) for x in xs], "global_features": gs, "Ps": Ps, "ns": ns,
           "gt_perm_mat": dd["gt_perm_mat"]}
    out2 = net.forward(dd2)
    for k in ("ds_mat", "perm_mat", "k_prob", "cls_prob"):
        assert torch.equal(out2[k], ref[k]), k
        assert torch.equal(out[k], ref[k]), k
    sdn = {k: v for k, v in net.state_dict().items()}
    orc = O.forward(pairs, sdn)
    ok = False
    try:
        rows = _k_gate(pairs, sdn, [ref], orc, exact_tol=K_EXACT)
        for r in (ref, out):
            assert (r["ds_mat"].cpu() - orc["ds_mat"]).abs().max() < 1e-4
        ok = True
    finally:
        if not ok or os.environ.get("FPM_DUMP_FEATS") == "1":
            _dump_feats("images_to_match_feats.npz", [torch.from_numpy(x) for x in xs_h],
                        [torch.from_numpy(g) for g in gs_h], Ps, ns)
    if os.environ.get("FPM_DUMP_FEATS") == "1":
        import json
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out",
                               "images_to_match_k.json"), "w") as f:
            json.dump(rows, f, indent=1)


K_GATE = 1e-4
K_EXACT = 2e-5       # the fp64 k chain: |k - k_fp64| (SplineConv + Kp are the only fp32 stages)


def _k_gate(pairs, sd, results, orc=None, gate=K_GATE, record=None, exact_tol=None):
    """k_prob of each device result against the exact (fp64 oracle) k of the same inputs: within
    ``gate`` beyond the fp32 reference's own deviation from it (max over the factorised and the
    explicit-pattern fp32 oracle) pair by pair (``gate=None``: record only); ``exact_tol``: also
    within that of the exact value itself.  Returns the per-pair deltas."""
    import oracle as O
    orc = orc if orc is not None else O.forward(pairs, sd)
    orx = O.forward(pairs, sd, explicit_pattern=True)
    o64 = O.forward(pairs, sd, dtype=torch.float64)
    k64 = o64["k_prob"]
    rows = []
    for b in range(len(pairs)):
        floor = max(abs(float(orc["k_prob"][b]) - float(k64[b])), abs(float(orx["k_prob"][b]) - float(k64[b])))
        row = {"pair": b, "ref32_floor": floor}
        for i, r in enumerate(results):
            d = abs(float(r["k_prob"][b]) - float(k64[b]))
            row["dev%d_k64" % i] = d
            row["dev%d_ref32" % i] = abs(float(r["k_prob"][b]) - float(orc["k_prob"][b]))
        rows.append(row)
    print("k gate", rows)
    if record is not None:
        record.extend(rows)
    for row in rows:
        for i in range(len(results)):
            d = row["dev%d_k64" % i]
            if gate is not None:
                assert d <= row["ref32_floor"] + gate, row
            if exact_tol is not None:
                assert d <= exact_tol, row
    return rows


def _cpu_image_pairs(B, n, seed):
    """Matcher inputs of an image batch from the seeded ResNet-18 on the CPU + the oracle front end
    (the same inputs in every run)."""
    import oracle as O
    from fpm.backbone import build_resnet18_split
    nl, el, _ = build_resnet18_split(0)
    nl.eval()
    el.eval()
    imgs, Ps, ns = _image_batch(B, n, seed)
    xs, gs = [], []
    with torch.no_grad():
        for side in range(2):
            nodes = nl(imgs[side])
            x, w = O.frontend_oracle.image_features(nodes, el(nodes), Ps[side], ns[side])
            xs.append(x.view(B, n, -1).numpy())
            gs.append(w.numpy())
    return _pairs_from_feats(xs, gs, Ps, ns)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_image_path_k_vs_exact(mode):
    """Both compute modes on image-derived matcher inputs (six image seeds, ragged n = 32 / 27 / 22)
    against the fp64 oracle on identical inputs: k within 1e-4 beyond the fp32 reference's own
    deviation from exact AND within 2e-5 of exact (the fp64 k chain, csrc/precise.hip, runs on these
    boxes in both modes); ss / ds_mat within 1e-4 of the fp32 oracle.

    Why the gate is anchored at the exact value: on these pairs the fp32 reference itself sits up to
    2e-4 from its own fp64 k (tools/kprob_diag.py) -- the fp32 rounding of any one stage after Kp
    moves k by up to ~6e-5 (tools/kprob_arith.py) -- so a device with any other summation order can
    not promise 1e-4 against one fp32 evaluation.  The features come from the seeded ResNet-18 on
    the CPU + the oracle front end (the same inputs every run); the MIOpen features of the device
    front end are gated in test_images_to_match_forward and test_image_fixture_k_vs_exact."""
    import fpm
    from fpm import params
    from fpm.batch import DeviceBatch
    import oracle as O
    import json
    sd = params.init_params(5)
    net = fpm.Net(regression=True, backbone=False, dtype=mode)
    net.load_state_dict(sd)
    rec = []
    for seed in range(8, 14):
        pairs = _cpu_image_pairs(3, 32, seed)
        bt = DeviceBatch.from_pairs(pairs, DEV)
        assert net._k_f64(bt)
        res = net.run(bt)
        orc = O.forward(pairs, sd)
        _k_gate(pairs, sd, [res], orc, record=rec, exact_tol=K_EXACT)
        for k in ("ss", "ds_mat"):
            assert (res[k].cpu() - orc[k]).abs().max() < 1e-4, k
        for r in rec[-3:]:
            r["seed"] = seed
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "image_k_vs_exact_%s.json" % mode), "w") as f:
        json.dump(rec, f, indent=1)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_image_fixture_k_vs_exact(mode):
    """The MIOpen-computed matcher inputs of a device image forward (tests/golden/image_feats_miopen.npz,
    captured on an MI355X by test_images_to_match_forward with FPM_DUMP_FEATS=1: the features the
    round-5 gate failed on are of this kind) through both modes: the k gate + 2e-5 of exact, ss /
    ds_mat within 1e-4 of the fp32 oracle."""
    import fpm
    from fpm import params
    from fpm.batch import DeviceBatch
    import oracle as O
    from conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "image_feats_miopen.npz"))
    pairs = _pairs_from_feats([z["x0"], z["x1"]], [z["g0"], z["g1"]], [z["P0"], z["P1"]], [z["n0"], z["n1"]])
    sd = params.init_params(5)
    net = fpm.Net(regression=True, backbone=False, dtype=mode)
    net.load_state_dict(sd)
    res = net.run(DeviceBatch.from_pairs(pairs, DEV))
    orc = O.forward(pairs, sd)
    _k_gate(pairs, sd, [res], orc, exact_tol=K_EXACT)
    for k in ("ss", "ds_mat"):
        assert (res[k].cpu() - orc[k]).abs().max() < 1e-4, k


@pytest.mark.gpu
@pytest.mark.parametrize("n", [96, 192])
@pytest.mark.parametrize("mode", ["f32", "bf16"])
def test_image_path_large_n(mode, n):
    """image-derived matcher inputs at n = 192 / 187 / 182 and 96 / 91 / 86 (padded
    boxes above the 64-keypoint thresholds: the bf16 mode runs its bf16 SplineConv products and split
    near-fp32 Kp, both modes the fp32 k chain -- the headline's kernels).  k is better conditioned
    here than at n = 32 (the fp32 reference within 3.6e-5 of exact at n = 192 and 6.4e-5 at n = 96,
    tools/kprob_diag.py --n; the bf16 products add <= 1e-5 at n = 192, tools/kprob_yround.py --n 192):
    the anchored k gate at both sizes, and at n = 192 the north-star gate as written (ss / ds_mat /
    k_prob within 1e-4 of the fp32 oracle); ss / ds_mat within 1e-4 at both."""
    import fpm
    from fpm import params
    from fpm.batch import DeviceBatch
    import oracle as O
    sd = params.init_params(5)
    net = fpm.Net(regression=True, backbone=False, dtype=mode)
    net.load_state_dict(sd)
    pairs = _cpu_image_pairs(3, n, 8)
    bt = DeviceBatch.from_pairs(pairs, DEV)
    assert not net._k_f64(bt) and net._sc_f32(bt) == (mode == "f32")
    res = net.run(bt)
    orc = O.forward(pairs, sd)
    _k_gate(pairs, sd, [res], orc)
    for k in (("ss", "ds_mat", "k_prob") if n >= 128 else ("ss", "ds_mat")):
        assert (res[k].cpu() - orc[k]).abs().max() < 1e-4, k


def _align_case(seed, B, n, Cn=256, Ce=512, hn=(15, 20), he=(8, 10)):
    """Random maps + keypoints incl. the frame's borders (the clamped-corner branch)."""
    g = torch.Generator().manual_seed(seed)
    nodes = torch.randn(B, Cn, *hn, generator=g, dtype=torch.float64)
    edges = torch.relu(torch.randn(B, Ce, *he, generator=g, dtype=torch.float64))
    P = torch.zeros(B, n, 2, dtype=torch.float32)
    ns = []
    for b in range(B):
        m = n - 3 * b
        P[b, :m, 0] = torch.rand(m, generator=g) * 320
        P[b, :m, 1] = torch.rand(m, generator=g) * 240
        P[b, 0] = torch.tensor([0.0, 0.0])          # corners / edges of the frame
        P[b, 1] = torch.tensor([319.9, 239.9])
        P[b, 2] = torch.tensor([3.0, 120.0])
        ns.append(m)
    return nodes, edges, P, torch.tensor(ns)


@pytest.mark.gpu
@pytest.mark.parametrize("channels_last", [False, True])
@pytest.mark.parametrize("case", ["golden", "c3"])
def test_feature_align_bwd_vs_autograd(channels_last, case):
    """fpm_feature_align_bwd (transpose of the bilinear gather, channel-norm backward, global
    max-pool gradient) against float64 autograd through the oracle front end (frontend_oracle,
    pinned by feature_align.npz) on the same fp32 maps: dnodes / dedges within 1e-5 of their scale."""
    from fpm import ops
    if case == "golden":
        z = _golden()
        nodes, edges, P, ns = z["nodes"].double(), z["edges"].double(), z["P"].float(), z["ns"]
    else:
        nodes, edges, P, ns = _align_case(4, 3, 48)
    nodes, edges = nodes.float().double(), edges.float().double()
    B, nmax = P.shape[:2]
    C = nodes.shape[1] + edges.shape[1]
    g = torch.Generator().manual_seed(77)
    dX = torch.randn(B, nmax, C, generator=g, dtype=torch.float64)
    dG = torch.randn(B, edges.shape[1], generator=g, dtype=torch.float64)
    nl, el = nodes.clone().requires_grad_(True), edges.clone().requires_grad_(True)
    X, G = FO.image_features(nl, el, P, ns)
    ((X * dX).sum() + (G * dG).sum()).backward()
    mf = torch.channels_last if channels_last else torch.contiguous_format
    nd = nodes.float().to(DEV).contiguous(memory_format=mf)
    ed = edges.float().to(DEV).contiguous(memory_format=mf)
    n32 = ns.to(torch.int32).to(DEV)
    Xd, Gd, ws = ops.feature_align(nd, ed, P.to(DEV), n32, keep_ws=True)
    dn, de = ops.feature_align_bwd(nd, ed, P.to(DEV), n32, ws, dX.float().reshape(B * nmax, C).to(DEV),
                                   dG.float().to(DEV))
    assert dn.is_contiguous(memory_format=mf) and de.is_contiguous(memory_format=mf)
    for got, ref in ((dn, nl.grad), (de, el.grad)):
        err = float((got.cpu().double() - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, err


@pytest.mark.gpu
def test_backbone_gradient_through_align_vs_oracle_front_end(deterministic_convs):
    """The backbone's parameter gradients through FeatureAlignFn (HIP forward + backward) against
    the same MIOpen backbone through the oracle's torch front end under autograd, for the same
    upstream gradients of the node rows and the global feature: within 1e-4 of each tensor's
    gradient scale (the two differ in the align stage's backward only)."""
    import fpm
    from fpm import train
    net = fpm.Net(regression=True, backbone=True)
    net.to(DEV).train()
    B, n = 2, 40
    imgs, Ps, ns = _image_batch(B, n, 13)
    img = imgs[0].to(DEV).contiguous(memory_format=torch.channels_last)
    g = torch.Generator().manual_seed(3)
    dX = torch.randn(B, n, 768, generator=g).to(DEV)
    dG = torch.randn(B, 512, generator=g).to(DEV)
    bb = [(k, p) for k, p in net.named_parameters() if k.startswith(("node_layers", "edge_layers"))]
    state = {k: v.clone() for k, v in net.state_dict().items()}
    grads = []
    for path in ("hip", "oracle", "hip"):
        net.load_state_dict(state)
        net.zero_grad(set_to_none=True)
        nodes = net.node_layers(img)
        edges = net.edge_layers(nodes)
        if path == "hip":
            X, G = train.FeatureAlignFn.apply(nodes, edges, Ps[0].to(DEV), ns[0].to(torch.int32).to(DEV), (320.0, 240.0))
            X = X.view(B, n, -1)
        else:
            X, G = FO.image_features(nodes, edges, Ps[0].to(DEV), ns[0])
        ((X * dX).sum() + (G * dG).sum()).backward()
        grads.append({k: p.grad.clone() for k, p in bb})
    # the library convolutions' weight-gradient reductions are not bitwise reproducible: two runs
    # of the same path spread by `noise`; the HIP and oracle paths must agree within that (or 1e-4)
    for k, _ in bb:
        ref = grads[1][k]
        scale = ref.abs().max().clamp(min=1e-30)
        err = float((grads[0][k] - ref).abs().max() / scale)
        noise = float((grads[0][k] - grads[2][k]).abs().max() / scale)
        assert err < max(1e-4, 3.0 * noise), (k, err, noise)


@pytest.mark.gpu
def test_train_backbone_gradient_end_to_end(deterministic_convs):
    """train.py stages 1 / 3 / 5: Net.forward in train mode on images (backbone under autograd,
    FeatureAlignFn, the matcher's HIP backward) gives every node_layers / edge_layers parameter a
    finite, non-zero gradient equal (1e-4 of each tensor's scale) to the run whose node rows are
    differentiated through the oracle's torch front end instead.  Run 2 feeds the matcher the HIP
    rows' values with the oracle rows' gradient path (x_hip + (x_oracle - x_oracle.detach())), so
    both runs see bit-identical matcher inputs: the tau = 0.01 Sinkhorn backwards would otherwise
    amplify the ~1e-7 difference of the two front ends' forward values to ~1e-2."""
    import fpm
    from fpm import params, train
    net = fpm.Net(regression=True, backbone=True)
    net.load_state_dict({**net.state_dict(), **params.init_params(5)})
    net.to(DEV).train()
    B, n = 2, 32
    imgs, Ps, ns = _image_batch(B, n, 11)
    gt = torch.zeros(B, n, n)
    for b in range(B):
        m = min(int(ns[0][b]), int(ns[1][b]))
        gt[b, torch.arange(m), torch.arange(m)] = 1.0
    n1, n2 = ns[0].tolist(), ns[1].tolist()

    def loss_of(out):
        # PermutationLoss + ks_loss (the classifier's perm mask is discrete: left out so both runs
        # see exactly the same differentiable graph)
        return train.permutation_loss(out["ds_mat"], gt, n1, n2) + out["ks_loss"]

    bb = [(k, p) for k, p in net.named_parameters() if k.startswith(("node_layers", "edge_layers"))]
    state = {k: v.clone() for k, v in net.state_dict().items()}
    runs = []
    for _ in range(2):          # twice: the library convolutions' run-to-run spread (`noise`)
        net.zero_grad(set_to_none=True)
        net.load_state_dict(state)
        out = net({"images": imgs, "Ps": Ps, "ns": ns, "gt_perm_mat": gt})
        loss_of(out).backward()
        runs.append({k: p.grad.clone() for k, p in bb})
    got = runs[0]
    for k, gr in got.items():
        assert torch.isfinite(gr).all() and gr.abs().max() > 0, k
    net.zero_grad(set_to_none=True)
    net.load_state_dict(state)                     # same BatchNorm running buffers as run 1
    xs, gs = [], []
    for side in range(2):
        img = imgs[side].to(DEV).contiguous(memory_format=torch.channels_last)
        nodes = net.node_layers(img)
        edges = net.edge_layers(nodes)
        X, G = FO.image_features(nodes.float(), edges.float(), Ps[side].to(DEV), ns[side])
        with torch.no_grad():
            Xh, Gh = net.image_features([imgs[side]], [Ps[side]], [ns[side]], DEV)
        xs.append(Xh[0].view_as(X) + (X - X.detach()))
        gs.append(Gh[0] + (G - G.detach()))
    out2 = net({"node_features": xs, "global_features": gs, "Ps": Ps, "ns": ns, "gt_perm_mat": gt})
    print("ds_mat run1 vs run2", float((out2["ds_mat"] - out["ds_mat"]).abs().max()))
    assert (out2["ds_mat"] - out["ds_mat"]).abs().max() < 1e-6
    loss_of(out2).backward()
    for k, p in bb:
        scale = p.grad.abs().max().clamp(min=1e-30)
        err = float((got[k] - p.grad).abs().max() / scale)
        noise = float((got[k] - runs[1][k]).abs().max() / scale)
        assert err < max(1e-4, 3.0 * noise), (k, err, noise)
