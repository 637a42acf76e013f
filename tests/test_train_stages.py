"""train.py's stage selection (``/root/reference/train.py:153-239``) against ``fpm.Net``.

The reference training script reads ``model.backbone_params`` (train.py:157,166),
``model.k_params_id`` (:158,186,213) and ``model.k_params`` (:172,196,209,219,227), set by
``feature_extractor.py:19`` and ``ngm.py:174-199``.  Two forms of the check:

* ``test_stage_block_restated``: the stage logic restated here (same membership rules and
  optimizer groups per stage), run on ``fpm.Net`` for stages 1-6 -- always runs;
* ``test_reference_stage_block_executes``: the reference script's own lines 153-239, read as text
  at run time from ``/root/reference`` (nothing of it is stored in this repo) and executed against
  ``fpm.Net``; skipped where the reference tree is absent (the GPU box).

Both check every stage's ``requires_grad`` set and optimizer parameter groups.
"""
import os

import pytest
import torch
import torch.optim as optim

import fpm

REF_TRAIN = "/root/reference/train.py"
LR, BACKBONE_LR, K_LR = 1e-3, 1e-5, 1e-4


def _groups(model):
    """Expected membership (ids): backbone, k regressor, match classifier, the rest."""
    bb = {id(p) for p in model.backbone_params}
    k = set(model.k_params_id)
    mc = {id(p) for p in model.match_cls.parameters()}
    allp = {id(p) for p in model.parameters()}
    return bb, k, mc, allp - bb - k - mc


def _expected_trainable(stage, model):
    bb, k, mc, other = _groups(model)
    return {1: bb | mc | other,            # k_params frozen, the rest left trainable
            2: k, 3: bb | k | mc | other, 4: k,
            5: bb | k | other,             # all but the match classifier
            6: mc}[stage]


def _check(model, stage, optimizer, optimizer_k):
    bb, k, mc, other = _groups(model)
    trainable = {id(p) for p in model.parameters() if p.requires_grad}
    assert trainable == _expected_trainable(stage, model), stage
    # optimizer: [other_params, backbone_params (BACKBONE_LR)] (train.py:164-167)
    g = optimizer.param_groups
    assert len(g) == 2
    assert {id(p) for p in g[0]["params"]} == other
    assert {id(p) for p in g[1]["params"]} == bb and g[1]["lr"] == BACKBONE_LR
    if stage in (2, 3, 4, 5):
        gk = optimizer_k.param_groups
        assert len(gk) == 3 and gk[0]["lr"] == K_LR
        assert {id(p) for grp in gk for p in grp["params"]} == k
        assert all(len(grp["params"]) > 0 for grp in gk)
    else:
        assert optimizer_k is None


def test_train_attributes_membership():
    model = fpm.Net(regression=True)
    names = {id(p): n for n, p in model.named_parameters()}
    bb, k, mc, other = _groups(model)
    assert bb and all(names[i].startswith(("node_layers.", "edge_layers.")) for i in bb)
    assert len(bb) == len(list(model.node_layers.parameters())) + len(list(model.edge_layers.parameters()))
    assert k and all(names[i].startswith(("encoder_k.", "final_row.", "final_col.")) for i in k)
    assert sum(n.startswith(("encoder_k.", "final_row.", "final_col.")) for n in names.values()) == len(k)
    assert any(names[i].startswith("message_pass_node_features.") for i in other)
    # k_params: three groups, re-iterable
    kp = model.k_params
    assert [len(g["params"]) for g in kp] == [len(list(m.parameters())) for m in
                                              (model.encoder_k, model.final_row, model.final_col)]
    assert {id(p) for g in model.k_params for p in g["params"]} == k
    # a matcher-only Net has no backbone parameters
    assert fpm.Net(regression=True, backbone=False).backbone_params == []


@pytest.mark.parametrize("stage", [1, 2, 3, 4, 5, 6])
def test_stage_block_restated(stage):
    """train.py:153-239 restated: freeze / unfreeze per stage and the optimizers it builds."""
    model = fpm.Net(regression=True)
    backbone_ids = [id(p) for p in model.backbone_params]
    k_params = model.k_params_id
    match_cls_ids = [id(p) for p in model.match_cls.parameters()]
    other_params = [p for p in model.parameters()
                    if id(p) not in k_params and id(p) not in backbone_ids and id(p) not in match_cls_ids]
    model_params = [{"params": other_params}, {"params": model.backbone_params, "lr": BACKBONE_LR}]
    optimizer_k = None
    if stage == 1:
        for grp in model.k_params:
            for p in grp["params"]:
                p.requires_grad = False
    elif stage in (2, 4):
        for _, p in model.named_parameters():
            p.requires_grad = id(p) in model.k_params_id
    elif stage == 3:
        for _, p in model.named_parameters():
            p.requires_grad = True
    elif stage == 5:
        for _, p in model.named_parameters():
            p.requires_grad = id(p) not in match_cls_ids
    elif stage == 6:
        for _, p in model.named_parameters():
            p.requires_grad = id(p) in match_cls_ids
    optimizer = optim.AdamW(model_params, lr=LR, weight_decay=1e-4)
    if stage in (2, 3, 4, 5):
        optimizer_k = optim.AdamW(model.k_params, lr=K_LR, weight_decay=1e-6)
    _check(model, stage, optimizer, optimizer_k)


def _reference_stage_block():
    with open(REF_TRAIN) as f:
        lines = f.read().split("\n")
    # train.py:153-239 (1-based, inclusive): the stage block up to the classifier optimizer
    block = lines[152:239]
    assert "backbone_ids" in block[4] and "optimizer_cls" in block[-1], "train.py moved"
    return "\n".join(l[4:] if l.startswith("    ") else l for l in block)


@pytest.mark.skipif(not os.path.exists(REF_TRAIN), reason="reference tree absent (GPU box)")
@pytest.mark.parametrize("stage", [1, 2, 3, 4, 5, 6])
def test_reference_stage_block_executes(stage):
    """The reference's own stage block, executed unchanged against fpm.Net."""
    src = _reference_stage_block()
    model = fpm.Net(regression=True)
    ns = {"model": model, "stage": stage, "optim": optim, "LR": LR, "BACKBONE_LR": BACKBONE_LR, "K_LR": K_LR,
          "print": lambda *a, **k: None, "torch": torch}
    exec(compile(src, REF_TRAIN + ":153-239", "exec"), ns)
    _check(model, stage, ns["optimizer"], ns["optimizer_k"])
