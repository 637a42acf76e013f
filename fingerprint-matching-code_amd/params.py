"""Parameter inventory of ``Net`` with the reference's state_dict names and shapes.

Names/shapes follow ``Net.__init__`` (``src/model/ngm.py:118-202``) and the third-party
modules it instantiates (PyG 1.6.3 ``SplineConv``/``SAGEConv``/``GCNConv``), so a reference
checkpoint loads by name+shape exactly as ``utils/models_sl.py:12-40`` does.  The ResNet-18
backbone (``node_layers.*``/``edge_layers.*``/``final_layers.*``) is out of scope.

``init_params`` draws a deterministic random initialisation in the reference's init ranges:
``nn.Linear`` default U(+-1/sqrt(fan_in)); SplineConv ``uniform(K*in, .)`` for weight/root/bias
(PyG 1.6.3 ``reset_parameters``); CrossSet mixed-score MLP U(+-10) (``afau.py:217-229``).
"""
import math
from collections import OrderedDict

import torch

from . import config as C

SPLINE_PREFIX = "message_pass_node_features.mp_network.convs"


def _u(gen, shape, bound):
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2.0 - 1.0).mul_(bound).float()


def _linear(sd, gen, name, out_f, in_f, bias=True):
    b = 1.0 / math.sqrt(in_f)
    sd[name + ".weight"] = _u(gen, (out_f, in_f), b)
    if bias:
        sd[name + ".bias"] = _u(gen, (out_f,), b)


def param_shapes():
    """Return an ordered name -> shape map (float parameters and buffers)."""
    return OrderedDict((k, tuple(v.shape)) for k, v in init_params(0).items())


def init_params(seed=0, perturb_norms=True):
    """Deterministic random-init state_dict of the matcher (backbone excluded).

    ``perturb_norms`` randomises the InstanceNorm affine parameters and the BatchNorm running
    statistics (the reference's fresh-module values are 1/0) so parity tests exercise them.
    """
    gen = torch.Generator().manual_seed(int(seed))
    sd = OrderedDict()
    d = C.NODE_FEATURE_DIM
    for i in range(2):
        p = "%s.%d" % (SPLINE_PREFIX, i)
        bound = 1.0 / math.sqrt(C.SPLINE_CELLS * d)
        sd[p + ".weight"] = _u(gen, (C.SPLINE_CELLS, d, d), bound)
        sd[p + ".root"] = _u(gen, (d, d), bound)
        sd[p + ".bias"] = _u(gen, (d,), bound)
        sd[p + ".kernel_size"] = torch.tensor([C.SPLINE_KERNEL, C.SPLINE_KERNEL], dtype=torch.long)
        sd[p + ".is_open_spline"] = torch.tensor([1, 1], dtype=torch.uint8)
    _linear(sd, gen, "vertex_affinity.A", d, C.GLOBAL_STATE_DIM)
    _linear(sd, gen, "edge_affinity.A", d, C.GLOBAL_STATE_DIM)
    for l in range(C.GNN_LAYER):
        cin = 1 if l == 0 else C.GNN_FEAT[l - 1] + C.SK_EMB
        cout = C.GNN_FEAT[l]
        p = "gnn_layer_%d" % l
        gb = math.sqrt(6.0 / (cin + cout))
        sd[p + ".conv.weight"] = _u(gen, (cin, cout), gb)          # GCNConv (never called, gnn.py:198)
        sd[p + ".conv.bias"] = torch.zeros(cout)
        _linear(sd, gen, p + ".conv2.lin_l", cout, cin)
        _linear(sd, gen, p + ".conv2.lin_r", cout, cin, bias=False)
        _linear(sd, gen, p + ".n_self_func.0", cout, cin)
        _linear(sd, gen, p + ".n_self_func.2", cout, cout)
        _linear(sd, gen, p + ".classifier", C.SK_EMB, cout)
    _linear(sd, gen, "classifier", 1, C.GNN_FEAT[-1] + C.SK_EMB)
    E, HD = C.AFAU_EMB, C.AFAU_HEADS * C.AFAU_QKV
    for blk in ("row", "col"):
        p = "encoder_k.layers.0.%s_encoding_block" % blk
        _linear(sd, gen, p + ".Wq", HD, E, bias=False)
        _linear(sd, gen, p + ".Wk", HD, E, bias=False)
        _linear(sd, gen, p + ".Wv", HD, E, bias=False)
        m = C.AFAU_MS_INIT
        sd[p + ".mixed_score_MHA.mix1_weight"] = _u(gen, (C.AFAU_HEADS, 2, C.AFAU_MS_HIDDEN), m)
        sd[p + ".mixed_score_MHA.mix1_bias"] = _u(gen, (C.AFAU_HEADS, C.AFAU_MS_HIDDEN), m)
        sd[p + ".mixed_score_MHA.mix2_weight"] = _u(gen, (C.AFAU_HEADS, C.AFAU_MS_HIDDEN, 1), m)
        sd[p + ".mixed_score_MHA.mix2_bias"] = _u(gen, (C.AFAU_HEADS, 1), m)
        _linear(sd, gen, p + ".multi_head_combine", E, HD)
        for k in (1, 2):
            q = p + ".add_n_normalization_%d.norm" % k
            if perturb_norms:
                sd[q + ".weight"] = 1.0 + _u(gen, (E,), 0.2)
                sd[q + ".bias"] = _u(gen, (E,), 0.2)
            else:
                sd[q + ".weight"] = torch.ones(E)
                sd[q + ".bias"] = torch.zeros(E)
        _linear(sd, gen, p + ".feed_forward.W1", C.AFAU_FF, E)
        _linear(sd, gen, p + ".feed_forward.W2", E, C.AFAU_FF)
    for head in ("final_row", "final_col"):
        _linear(sd, gen, head + ".0", C.REG_HIDDEN, C.UNIV_SIZE)
        _linear(sd, gen, head + ".2", 1, C.REG_HIDDEN)
    cin = 1
    for idx, ch in zip((0, 4), C.CLS_CHANNELS):
        bnd = 1.0 / math.sqrt(cin * 9)
        sd["match_cls.conv.%d.weight" % idx] = _u(gen, (ch, cin, 3, 3), bnd)
        sd["match_cls.conv.%d.bias" % idx] = _u(gen, (ch,), bnd)
        bn = "match_cls.conv.%d" % (idx + 2)
        if perturb_norms:
            sd[bn + ".weight"] = 1.0 + _u(gen, (ch,), 0.2)
            sd[bn + ".bias"] = _u(gen, (ch,), 0.2)
            sd[bn + ".running_mean"] = _u(gen, (ch,), 0.1)
            sd[bn + ".running_var"] = 1.0 + _u(gen, (ch,), 0.5)
        else:
            sd[bn + ".weight"] = torch.ones(ch)
            sd[bn + ".bias"] = torch.zeros(ch)
            sd[bn + ".running_mean"] = torch.zeros(ch)
            sd[bn + ".running_var"] = torch.ones(ch)
        sd[bn + ".num_batches_tracked"] = torch.tensor(0, dtype=torch.long)
        cin = ch
    _linear(sd, gen, "match_cls.fc", 1, C.CLS_CHANNELS[-1])
    return sd
