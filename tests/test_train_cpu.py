"""CPU side of the training backward: the oracle's training-mode forward is
differentiable end to end (it is the gradient reference of tests/test_train.py), its
PermutationLoss restatement matches the reference formula, and the product's AFA-U replay
(``fpm.afau_torch``, used by the backward) equals the oracle's AFA-U on the same inputs."""
import torch
import torch.nn.functional as F

from fpm import afau_torch, params, synth
import oracle as O


def test_oracle_training_step_differentiable():
    sd = params.init_params(3)
    pairs = synth.make_batch(4, 2, 16)
    sdl = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running_" not in k else v.clone())
           for k, v in sd.items()}
    gt = torch.zeros(2, 16, 16)
    gt[:, torch.arange(16), torch.arange(16)] = 1
    out = O.forward(pairs, sdl, training=True, gt_perm=gt, labels=torch.tensor([1.0, 0.0]))
    loss = O.permutation_loss(out["ds_mat"], gt, [16, 16], [16, 16]) + out["ks_loss"] + out["cls_loss"]
    loss.backward()
    got = [k for k, v in sdl.items() if v.requires_grad and v.grad is not None]
    assert len(got) >= 60
    for k in got:
        assert torch.isfinite(sdl[k].grad).all(), k
    # encoder / head grads come from ks_loss only (ss detached): the GNN gets none from it
    assert sdl["encoder_k.layers.0.row_encoding_block.Wk.weight"].grad is not None
    # running statistics moved (train-mode BatchNorm)
    assert not torch.equal(sdl["match_cls.conv.2.running_mean"], sd["match_cls.conv.2.running_mean"])


def test_permutation_loss_formula():
    g = torch.Generator().manual_seed(0)
    ds = torch.rand(3, 6, 7, generator=g).clamp(1e-3, 1 - 1e-3)
    gt = (torch.rand(3, 6, 7, generator=g) > 0.8).float()
    n1, n2 = [6, 4, 5], [7, 6, 3]
    ref = sum(-(gt[b, :n1[b], :n2[b]] * ds[b, :n1[b], :n2[b]].log()
                + (1 - gt[b, :n1[b], :n2[b]]) * (1 - ds[b, :n1[b], :n2[b]]).log()).sum() for b in range(3)) / sum(n1)
    assert abs(float(O.permutation_loss(ds, gt, n1, n2)) - float(ref)) < 1e-5
    from fpm import train
    assert abs(float(train.permutation_loss(ds, gt, n1, n2)) - float(ref)) < 1e-5


def test_afau_replay_equals_oracle():
    sd = params.init_params(5)
    g = torch.Generator().manual_seed(1)
    n1, n2 = torch.tensor([12, 9]), torch.tensor([10, 12])
    ss = torch.rand(2, 12, 12, generator=g, dtype=torch.float64)
    for b in range(2):
        ss[b, n1[b]:] = 0
        ss[b, :, n2[b]:] = 0
    sdd = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    ref = O.afau_ks(ss, n1, n2, sdd)
    ours = afau_torch.afau_ks(ss, n1, n2, lambda k: sdd[k])
    assert (ref - ours).abs().max() < 1e-12


def test_afau_replay_gradients_equal_oracle():
    """The training backward's AFA-U gradients are autograd through fpm.afau_torch: in float64 at
    the same ss they equal autograd through the oracle's AFA-U (same formulation)."""
    sd = params.init_params(6)
    g = torch.Generator().manual_seed(2)
    n1, n2 = torch.tensor([12, 9, 12]), torch.tensor([10, 12, 12])
    ss = torch.rand(3, 12, 12, generator=g, dtype=torch.float64)
    names = [k for k in sd if k.startswith(afau_torch.AFAU_PARAM_PREFIXES)]
    a = {k: sd[k].double().clone().requires_grad_(True) for k in names}
    b = {k: sd[k].double().clone().requires_grad_(True) for k in names}
    sdd = {k: v.double() if v.is_floating_point() else v for k, v in sd.items()}
    sdd.update(b)
    w = torch.tensor([0.3, -1.0, 0.7], dtype=torch.float64)
    (afau_torch.afau_ks(ss, n1, n2, lambda k: a[k]) * w).sum().backward()
    (O.afau_ks(ss, n1, n2, sdd) * w).sum().backward()
    for k in names:
        ga, gb = a[k].grad, b[k].grad
        if gb is None:
            assert ga is None or float(ga.abs().max()) == 0.0, k
            continue
        assert float((ga - gb).abs().max()) <= 1e-9 * max(1.0, float(gb.abs().max())), k
