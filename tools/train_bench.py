"""Training-step throughput: one step = Net.forward in train mode +
PermutationLoss(ds_mat) + ks_loss + cls_loss, backward, AdamW step (training_loop.py:23-70 with
stage 3's all-parameters-trainable grouping), on B synthetic pairs of n-keypoint Delaunay graphs.

    python tools/train_bench.py [--batch 64] [--n 256] [--dtype bf16] [--steps 5] [--warmup 2]
                                [--cpu-pairs 2]

Prints one JSON line: pairs/s, ms per step and its forward / backward / optimizer split (HIP
events), and the CPU oracle's training step (autograd) on a bounded sample beside it.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-pairs", type=int, default=2)
    ap.add_argument("--no-regression", action="store_true", help="Net(regression=False): no AFA-U")
    args = ap.parse_args()
    import torch
    import fpm
    from fpm import params, synth, train
    from fpm.batch import DeviceBatch

    dev = torch.device("cuda", 0)
    sd = params.init_params(1)
    pairs = synth.make_batch(3, args.batch, args.n)
    bt = DeviceBatch.from_pairs(pairs, dev)
    B, n = args.batch, args.n
    gt = torch.zeros(B, n, n, device=dev)
    gt[:, torch.arange(n), torch.arange(n)] = 1.0
    label = (torch.arange(B, device=dev) % 2).float()
    net = fpm.Net(regression=not args.no_regression, backbone=False, dtype=args.dtype)
    net.load_state_dict(sd)
    net.to(dev).train()
    opt = torch.optim.AdamW([p for p in net.parameters() if p.requires_grad], lr=1e-4, weight_decay=1e-4)
    ns = [bt.n_host[0], bt.n_host[1]]

    def step(ev=None):
        opt.zero_grad(set_to_none=True)
        if ev:
            ev[0].record()
        out = net({"fpm_batch": bt, "gt_perm_mat": gt, "label": label})
        loss = train.permutation_loss(out["ds_mat"], gt, ns[0], ns[1]) + out["ks_loss"] + out["cls_loss"]
        if ev:
            ev[1].record()
        loss.backward()
        if ev:
            ev[2].record()
        opt.step()
        if ev:
            ev[3].record()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        loss = step(evs[k])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    fwd = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
    bwd = sum(e[1].elapsed_time(e[2]) for e in evs) / args.steps
    optm = sum(e[2].elapsed_time(e[3]) for e in evs) / args.steps
    res = {"metric": "training pairs/sec (forward + backward + AdamW)", "value": B / dt, "unit": "pairs/s",
           "ms_per_step": dt * 1e3, "forward_ms": fwd, "backward_ms": bwd, "optimizer_ms": optm,
           "batch": B, "n": n, "dtype": args.dtype, "loss": float(loss)}
    if args.cpu_pairs > 0:
        import oracle as O
        cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), len(os.sched_getaffinity(0))))
        torch.set_num_threads(cores)
        cp = pairs[:args.cpu_pairs]
        g = gt[:args.cpu_pairs].cpu()
        sdl = {k: (v.clone().requires_grad_(True) if v.is_floating_point() and "running_" not in k else v.clone())
               for k, v in sd.items()}
        t = time.perf_counter()
        r = O.forward(cp, sdl, training=True, gt_perm=g, labels=label[:args.cpu_pairs].cpu())
        l = O.permutation_loss(r["ds_mat"], g, [n] * len(cp), [n] * len(cp)) + r["ks_loss"] + r["cls_loss"]
        l.backward()
        ct = time.perf_counter() - t
        res["cpu_baseline"] = {"value": len(cp) / ct, "unit": "pairs/s", "cores": cores, "kind": "port",
                               "sample": "%d pairs, n=%d, fp32 oracle forward + autograd backward" % (len(cp), n)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
