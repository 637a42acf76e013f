"""C-ABI library: loads, exports every symbol include/fpm.h declares; host-side LSA parity
(CPU only — no device call is made here)."""
import ctypes
import os
import re

import numpy as np
import pytest
import scipy.optimize as opt
import torch

import fpm  # noqa: F401
from fpm import _lib, params

from conftest import REPO


def _declared():
    src = open(os.path.join(REPO, "include", "fpm.h")).read()
    return sorted(set(re.findall(r"\b(fpm_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported():
    lib = _lib.load()
    names = _declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # every binding in _lib.SIGNATURES is declared in the header and vice versa
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_error_channel():
    lib = _lib.load()
    with pytest.raises(_lib.FpmError, match="n1max/n2max > 2048"):
        _lib.call("fpm_sinkhorn_log_fwd", None, 0, 0, 1, None, 0, 0, 1, None, None, 1, 3000, 300, 10, 0.01, 1, None)
    assert b"2048" in lib.fpm_last_error()
    with pytest.raises(_lib.FpmError, match="strides"):
        _lib.call("fpm_sinkhorn_log_fwd", None, 0, 2, 2, None, 0, 0, 1, None, None, 1, 30, 30, 10, 0.01, 1, None)


def test_sinkhorn_workspace_contract():
    """fpm_sinkhorn_ws_bytes (host arithmetic only): no workspace for boxes <= 256 (register
    kernels), a 16-B-multiple counter block + two exchange slots per sibling above; a too-small
    workspace is refused before any launch."""
    lib = _lib.load()
    assert lib.fpm_sinkhorn_ws_bytes(64, 256, 256) == 0
    assert lib.fpm_sinkhorn_ws_bytes(0, 512, 512) == 0
    b1, b8 = lib.fpm_sinkhorn_ws_bytes(1, 512, 300), lib.fpm_sinkhorn_ws_bytes(8, 512, 300)
    assert 0 < b1 < b8 and b1 % 16 == 0 and b8 % 16 == 0
    assert lib.fpm_sinkhorn_ws_bytes(8, 300, 512) == b8               # the larger side sets the slot
    with pytest.raises(_lib.FpmError, match="workspace"):
        _lib.call("fpm_sinkhorn_log_fwd_ws", None, 0, 512, 1, None, 0, 512, 1, None, None, 8, 512, 300, 10,
                  0.01, 1, ctypes.c_void_p(16), b8 - 16, None)


def test_wrong_result_probe_gated(monkeypatch):
    """the 'gnn_mlp_off' timing probe (wrong GNN results) is refused by fpm_set_tuning
    unless FPM_TIMING_PROBES=1, and Net.run refuses to produce outputs while it is on."""
    from fpm import ops
    monkeypatch.delenv("FPM_TIMING_PROBES", raising=False)
    with pytest.raises(_lib.FpmError, match="timing probe"):
        ops.set_tuning("gnn_mlp_off", 1)
    assert ops.timing_probes_on() == []
    monkeypatch.setenv("FPM_TIMING_PROBES", "1")
    try:
        ops.set_tuning("gnn_mlp_off", 1)
        assert ops.timing_probes_on() == ["gnn_mlp_off"]
        net = fpm.Net(regression=True, backbone=False)
        with pytest.raises(_lib.FpmError, match="timing probe"):
            net.run(None)
    finally:
        ops.set_tuning("gnn_mlp_off", 0)
    assert ops.timing_probes_on() == []


def test_cpu_tensor_rejected():
    from fpm import ops
    with pytest.raises(_lib.FpmError, match="CPU tensor"):
        ops.cast_bf16(torch.zeros(4))


def _lsa_ref(s, n1, n2):
    r, c = opt.linear_sum_assignment(s[:n1, :n2] * -1)
    a = -np.ones(s.shape[0], np.int32)
    a[r] = c
    return a


@pytest.mark.parametrize("mode", ["rand", "ties", "zeros", "sparse"])
def test_lsa_host_matches_scipy(mode):
    from fpm import ops
    rng = np.random.default_rng({"rand": 1, "ties": 2, "zeros": 3, "sparse": 4}[mode])
    B, n1max, n2max = 24, 37, 41
    s = np.zeros((B, n1max, n2max), np.float32)
    n1 = rng.integers(1, n1max + 1, B).astype(np.int32)
    n2 = rng.integers(1, n2max + 1, B).astype(np.int32)
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
    out = ops.lsa_batch_host(torch.from_numpy(s), torch.from_numpy(n1), torch.from_numpy(n2), nthreads=4)
    for b in range(B):
        np.testing.assert_array_equal(out[b].numpy(), _lsa_ref(s[b], n1[b], n2[b]))


def test_lsa_host_golden():
    """Same assignment as the reference's utils/hungarian on its golden case."""
    from fpm import ops
    from conftest import GOLDEN
    z = np.load(os.path.join(GOLDEN, "hungarian_greedy.npz"))
    s = torch.from_numpy(z["s"])
    a = ops.lsa_batch_host(s, torch.from_numpy(z["n1"]), torch.from_numpy(z["n2"]))
    x = np.zeros_like(z["x"])
    for b in range(x.shape[0]):
        for r, c in enumerate(a[b].tolist()):
            if c >= 0:
                x[b, r, c] = 1
    np.testing.assert_array_equal(x, z["x"])


def test_state_dict_names():
    """Parameter names/shapes follow Net.__init__ (ngm.py:118-202) incl. PyG/torch module names."""
    net = fpm.Net(regression=True, backbone=False)
    sd = net.state_dict()
    assert sd["message_pass_node_features.mp_network.convs.0.weight"].shape == (25, 768, 768)
    assert sd["message_pass_node_features.mp_network.convs.1.root"].shape == (768, 768)
    assert sd["vertex_affinity.A.weight"].shape == (768, 1024)
    assert sd["gnn_layer_0.conv2.lin_l.weight"].shape == (16, 1)
    assert sd["gnn_layer_2.conv2.lin_r.weight"].shape == (16, 17)
    assert sd["gnn_layer_1.n_self_func.2.weight"].shape == (16, 16)
    assert sd["classifier.weight"].shape == (1, 17)
    p = "encoder_k.layers.0.row_encoding_block."
    assert sd[p + "mixed_score_MHA.mix1_weight"].shape == (16, 2, 16)
    assert sd[p + "multi_head_combine.weight"].shape == (600, 256)
    assert sd[p + "feed_forward.W1.weight"].shape == (256, 600)
    assert sd["final_row.0.weight"].shape == (8, 600)
    assert sd["match_cls.conv.4.weight"].shape == (32, 16, 3, 3)
    assert sd["match_cls.conv.6.running_var"].shape == (32,)
    net2 = fpm.Net(regression=True, backbone=False, seed=3)
    net2.load_state_dict(sd)
    assert torch.equal(net2.state_dict()["vertex_affinity.A.bias"], sd["vertex_affinity.A.bias"])


def test_default_net_carries_backbone():
    """Net() like the reference's (ngm.py:118, 226-249): regression off, ResNet-18 backbone
    parameters under the reference names; a full reference-named state_dict loads strictly."""
    from fpm.backbone import backbone_state_dict
    net = fpm.Net()
    assert not net.regression
    sd = net.state_dict()
    assert sd["node_layers.0.weight"].shape == (64, 3, 7, 7)
    assert sd["edge_layers.0.1.bn2.running_var"].shape == (512,)
    assert "vertex_affinity.A.weight" in sd
    full = dict(params.init_params(2))
    full.update(backbone_state_dict(2))
    net.load_state_dict(full)
    assert torch.equal(net.state_dict()["node_layers.4.0.conv1.weight"], full["node_layers.4.0.conv1.weight"])
    bare = fpm.Net(backbone=False)
    assert not any(k.startswith(("node_layers.", "edge_layers.")) for k in bare.state_dict())
