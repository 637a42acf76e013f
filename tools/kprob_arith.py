"""Which stage's fp32 ARITHMETIC moves k_prob on image-derived matcher inputs.

fp64 oracle forward with exactly one stage evaluated in fp32 (inputs, weights and every operation
of that stage in fp32; its output widened back to fp64).  kprob_sources.py rounds one stage's
OUTPUT only; this probe charges each stage its full fp32 arithmetic.  Printed per pair: |k - k64|
for each stage and for the whole fp32 forward.

    python tools/kprob_arith.py [--seeds 8,9,10] [--B 3] [--n 32]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def _f32(a):
    if torch.is_tensor(a) and a.is_floating_point():
        return a.float()
    if isinstance(a, (list, tuple)):
        return type(a)(_f32(x) for x in a)
    return a


def _f64(a):
    if torch.is_tensor(a) and a.is_floating_point():
        return a.double()
    if isinstance(a, tuple):
        return tuple(_f64(x) for x in a)
    return a


STAGES = ("sconv", "kp", "gnn0", "gnn1", "gnn2", "gnn_sk", "gnn_lin", "gnn_agg", "gnn_x1", "gnn_x1r", "gnn_z",
          "readout", "finalsk", "afau")


def gnn_layer_split(x, sd, l, agg_fn, n1max, n2max, n1b, n2b, prec):
    """ngm_oracle.gnn_layer with per-operation precision: prec[op] in {32, 64} for op in agg (the
    pattern mean), x1 (lin_l / lin_r / MLP arithmetic), x1r (x1 stored in fp32 only), z (the
    classifier)."""
    import torch.nn.functional as F
    from oracle import ngm_oracle as NO
    p = "gnn_layer_%d" % l
    dt = lambda op: torch.float32 if prec.get(op) == 32 else torch.float64
    g = lambda k, op: sd[p + k].to(dt(op))
    agg = agg_fn(x.to(dt("agg"))).double()
    t = dt("x1")
    xa, xx = agg.to(t), x.to(t)
    x1 = F.linear(xa, g(".conv2.lin_l.weight", "x1"), g(".conv2.lin_l.bias", "x1")) + \
        F.linear(xx, g(".conv2.lin_r.weight", "x1"))
    h = F.relu(F.linear(xx, g(".n_self_func.0.weight", "x1"), g(".n_self_func.0.bias", "x1")))
    x1 = (x1 + F.relu(F.linear(h, g(".n_self_func.2.weight", "x1"), g(".n_self_func.2.bias", "x1")))).double()
    if prec.get("x1r") == 32:
        x1 = x1.float().double()
    z = F.linear(x1.to(dt("z")), g(".classifier.weight", "z"), g(".classifier.bias", "z")).double()
    Z = z.t().reshape(1, n2max, n1max).transpose(1, 2)
    S = NO.pygm_sinkhorn(Z, [n1b], [n2b], dummy_row=True, max_iter=NO.GNN_SK_ITER, tau=NO.TAU)
    x5 = S.transpose(2, 1).contiguous().reshape(1, 1, n1max * n2max).permute(0, 2, 1)[0]
    return torch.cat([x1, x5], dim=-1)


def run(pairs, sd, stage):
    import oracle as O
    from oracle import ngm_oracle as NO
    orig = {k: getattr(NO, k) for k in ("siamese_sconv", "affinity", "gnn_layer", "readout", "pygm_sinkhorn",
                                         "afau_ks")}

    def in32(name, cond=lambda *a, **k: True):
        f = orig[name]

        def g(*a, **k):
            if not cond(*a, **k):
                return f(*a, **k)
            return _f64(f(*_f32(a), **{kk: _f32(v) for kk, v in k.items()}))
        return g

    if stage == "sconv":
        NO.siamese_sconv = in32("siamese_sconv")
    elif stage == "kp":
        NO.affinity = in32("affinity")
    elif stage.startswith("gnn") and stage[3:].isdigit():
        l = int(stage[3:])
        NO.gnn_layer = in32("gnn_layer", lambda x, sd_, ll, *a, **k: ll == l)
    elif stage == "gnn_sk":
        NO.pygm_sinkhorn = in32("pygm_sinkhorn", lambda *a, **k: k.get("max_iter") == NO.GNN_SK_ITER)
    elif stage == "gnn_lin":
        # the layer's aggregation + linear maps in fp32, its Sinkhorn in fp64
        fl = orig["gnn_layer"]
        sk = orig["pygm_sinkhorn"]

        def gl(x, sd_, l, agg_fn, *a, **k):
            NO.pygm_sinkhorn = lambda s, *aa, **kk: sk(s.double(), *aa, **kk)
            try:
                y = fl(x.float(), sd_, l, lambda t: agg_fn(t.float()), *a, **k)
            finally:
                NO.pygm_sinkhorn = sk
            return y.double()
        NO.gnn_layer = gl
    elif stage in ("gnn_agg", "gnn_x1", "gnn_x1r", "gnn_z"):
        NO.gnn_layer = lambda x, sd_, l, agg_fn, *a, **k: gnn_layer_split(x, sd_, l, agg_fn, *a,
                                                                             prec={stage[4:]: 32})
    elif stage == "readout":
        NO.readout = in32("readout")
    elif stage == "finalsk":
        NO.pygm_sinkhorn = in32("pygm_sinkhorn", lambda *a, **k: k.get("max_iter") == NO.SK_ITER)
    elif stage == "afau":
        NO.afau_ks = in32("afau_ks")
    try:
        return O.forward(pairs, sd, dtype=torch.float64 if stage != "all32" else torch.float32)
    finally:
        for k, v in orig.items():
            setattr(NO, k, v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="8,9,10,11,12,13")
    ap.add_argument("--B", type=int, default=3)
    ap.add_argument("--n", type=int, default=32)
    args = ap.parse_args()
    from fpm import params
    from kprob_diag import image_pairs
    torch.set_num_threads(max(1, len(os.sched_getaffinity(0))))
    sd = params.init_params(5)
    worst = {}
    for seed in [int(s) for s in args.seeds.split(",")]:
        pairs = image_pairs(args.B, args.n, seed)
        k64 = run(pairs, sd, "none")["k_prob"]
        row = {}
        for st in STAGES + ("all32",):
            d = (run(pairs, sd, st)["k_prob"].double() - k64).abs()
            row[st] = d
            worst[st] = max(worst.get(st, 0.0), float(d.max()))
        for b in range(args.B):
            print("seed %2d pair %d  " % (seed, b) + " ".join("%s %.1e" % (st, float(row[st][b])) for st in row),
                  flush=True)
    print("worst: " + " ".join("%s %.1e" % kv for kv in worst.items()))


if __name__ == "__main__":
    main()
