"""Which bf16 rounding of the SplineConv moves k_prob on image-derived inputs (CPU; VERDICT r4 item 1,
round-5 follow-up).  The bf16 device mode rounds the product GEMM's OPERANDS (node rows x, cell
weights W) to bf16 and stores the (node, cell) product rows Y in bf16 before the fp32 4-corner sum;
tools/kprob_sources.py's bf16src probe rounded the operands only.  Here the oracle forward runs with

  ops     bf16 x and W in the products (fp32 accumulation), Y kept fp32
  ops+Y   the same, Y rounded to bf16 (the device's bf16 mode)
  Y       fp32 operands, Y rounded to bf16
  ops+Y1  bf16 operands, Y rounded in layer 1 only (layer 2's Y fp32)

and reports, per pair, |k - k64| beyond the fp32 oracle's own |k32 - k64| (the image-path gate's
"excess"), on the test's image seeds (tests/test_frontend.py::_image_batch, CPU backbone).

    python tools/kprob_yround.py [--seeds 8,9,10,11,12,13] [--n 32]
"""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="8,9,10,11,12,13")
    ap.add_argument("--n", type=int, default=32)
    args = ap.parse_args()
    import oracle as O
    from oracle import ngm_oracle as NO
    from fpm import params
    from kprob_diag import image_pairs
    sd = params.init_params(5)
    bf = lambda t: t.to(torch.bfloat16).to(t.dtype)
    o_sc = NO.spline_conv
    layer = [0]

    def make_sc(ops_bf, y_bf, y_layers):
        def sc(x, edge_index, pseudo, weight, root, bias):
            dt = x.dtype
            n, d = x.shape
            basis, wi = NO.spline_basis(pseudo)
            basis = basis.to(dt)
            K = weight.shape[0]
            xo = bf(x) if ops_bf else x
            W = torch.cat([weight.to(dt), root.to(dt)[None]])          # root as cell K (device layout)
            Wo = bf(W) if ops_bf else W
            Y = (xo @ Wo.permute(1, 0, 2).reshape(d, -1)).view(n, K + 1, -1)
            if y_bf and layer[0] in y_layers:
                Y = bf(Y)
            layer[0] += 1
            src, dst = edge_index[0].long(), edge_index[1].long()
            msg = None
            for s in range(4):
                t = basis[:, s:s + 1] * Y[src, wi[:, s]]
                msg = t if msg is None else msg + t
            out = torch.zeros(n, Y.shape[-1], dtype=dt)
            if src.numel():
                out = out.scatter_reduce(0, dst[:, None].expand(-1, Y.shape[-1]), msg, reduce="amax",
                                         include_self=False)
            return out + Y[:, K] + bias.to(dt)
        return sc

    variants = {"ops": (True, False, ()), "ops+Y": (True, True, (0, 1)), "Y": (False, True, (0, 1)),
                "ops+Y1": (True, True, (0,))}
    worst = {v: 0.0 for v in variants}
    for seed in map(int, args.seeds.split(",")):
        pairs = image_pairs(3, args.n, seed)
        k32 = O.forward(pairs, sd)["k_prob"].double()
        k64 = O.forward(pairs, sd, dtype=torch.float64)["k_prob"]
        floor = (k32 - k64).abs()
        line = ["seed %d floor %s" % (seed, ["%.1e" % float(f) for f in floor])]
        for name, (ob, yb, yl) in variants.items():
            # siamese_sconv calls spline_conv twice per side: layers counted mod 2
            def sc_layer(*a, _f=make_sc(ob, yb, yl), **k):
                r = _f(*a, **k)
                layer[0] %= 2
                return r
            NO.spline_conv = sc_layer
            try:
                layer[0] = 0
                kv = O.forward(pairs, sd)["k_prob"].double()
            finally:
                NO.spline_conv = o_sc
            ex = (kv - k64).abs() - floor
            worst[name] = max(worst[name], float(ex.max()))
            line.append("%s %s" % (name, ["%.1e" % float(e) for e in ex]))
        print("  ".join(line), flush=True)
    print("max excess over the fp32 oracle's own deviation:", {k: "%.2e" % v for k, v in worst.items()})


if __name__ == "__main__":
    main()
