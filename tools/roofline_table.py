"""Per-kernel roofline table of one bench run from its rocprofv3 kernel statistics.

    python tools/roofline_table.py STATS.csv --forwards F [--n 256] [--pairs 1024] [--out profiles/rNN_roofline]

STATS.csv is ``rocprofv3 --kernel-trace --stats`` output (``*_kernel_stats.csv``) of a command that
ran F full forwards of ``--pairs`` pairs of n-keypoint graphs (bench.py: warmup + 2 x steps + 1
isolated forward).  For each hot kernel: algorithmic bytes (or FLOPs) per pair and per call, times
the pairs the run processed, divided by the kernel's summed duration -> achieved GB/s (TFLOP/s)
and the fraction of the MI355X peak (HBM 8 TB/s; dense bf16 MFMA 2.5 PFLOP/s, fp32 157.3 TFLOP/s).
Durations are kernel-trace durations in the pipelined forward (two compute streams share the CUs),
so they include the co-running kernels' share of the machine: a lower bound on what the kernel
reaches alone.

Algorithmic work per pair at n keypoints, N = n^2 association nodes, E directed edges per graph
(DESIGN.md §3):
  gnn_layer_kernel<17>  reads X (17 N fp32), writes 16 channels + z (17 N) on layers 1, the fused
                        vpart + z (2 N) on the last layer: (17 + 17) and (17 + 2) x 4N B
  gnn_layer_kernel<1>   reads 1 N, writes 17 N: 18 x 4N B
  sinkhorn_*            reads s and writes the result: 2 x 4N B per call, 4 calls
  soft_topk_kernel      reads ss, writes ds_mat: 2 x 4N B
  combine_kernel        the side-layer's distinct product rows (rows/node x n x 768 bf16), the
                        output rows (n x 768 bf16 + fp32 on layer 2), residual read on layer 2
  topk_select_kernel    reads ds_mat at the matches, writes perm + lsa (2 x 4N B)
  affinity GEMM         2 n^2 768 FLOP (bf16 MFMA)
  product GEMM          2 rows 768^2 FLOP per side-layer (bf16 MFMA)
"""
import argparse
import csv
import json
import os

HBM = 8000.0          # GB/s
BF16 = 2500.0         # TFLOP/s dense
F32 = 157.3


def work(n, E, rows_per_node):
    N = n * n
    f4 = 4.0 * N
    spline_rows = rows_per_node * n
    comb_l1 = spline_rows * 768 * 2 + n * 768 * 2                      # product rows + bf16 output
    comb_l2 = spline_rows * 768 * 2 + n * 768 * (2 + 4) + n * 768 * 4    # + fp32 output + residual read
    return [
        # (match substring, kind, per-pair work over all calls of one forward, calls per pair, note)
        ("gnn_layer_kernel<17", "bytes", (17 + 17) * f4 + (17 + 2) * f4, 2, "layers 2-3: X in, 16 ch + z / vpart + z out"),
        ("gnn_layer_kernel<1,", "bytes", 18 * f4, 1, "layer 1: 1 ch in, 16 ch + z out"),
        ("sinkhorn_reg_kernel", "bytes", 4 * 2 * f4, 4, "3 GNN Sinkhorns (20 it) + final (10 it), s in, out out"),
        ("sinkhorn_lform_kernel", "bytes", 4 * 2 * f4, 4, "3 GNN Sinkhorns (20 it) + final (10 it), s in, out out"),
        ("sinkhorn_stream_kernel", "bytes", 4 * 2 * f4, 4, "same, n > 256"),
        ("soft_topk_kernel", "bytes", 2 * f4, 1, "ss in, ds_mat out"),
        ("combine_kernel", "bytes", 2 * (comb_l1 + comb_l2), 4, "2 sides x 2 layers: product rows + output (+ residual)"),
        ("topk_select_kernel", "bytes", 2 * f4, 1, "perm + lsa matrices out"),
        ("gemm_big_kernel<128, 3", "flops_bf16", 2.0 * N * 768, 1, "vertex affinity Kp (softplus epilogue)"),
        ("gemm_phase_kernel<0", "flops_bf16", 2 * 2 * 2.0 * spline_rows * 768 * 768, 4, "SplineConv (node, cell) products"),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("--forwards", type=int, required=True)
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--edges", type=float, default=1501.2, help="directed edges per graph (bench: E/graph)")
    ap.add_argument("--rows-per-node", type=float, default=9.7, help="spline product rows per node and layer")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats)))
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    pairs = a.forwards * a.pairs
    table = []
    for key, kind, per_pair, calls, note in work(a.n, a.edges, a.rows_per_node):
        hit = [r for r in rows if key in r["Name"]]
        if not hit:
            continue
        ns = sum(float(r["TotalDurationNs"]) for r in hit)
        cnt = sum(int(r["Calls"]) for r in hit)
        amount = per_pair * pairs
        if kind == "bytes":
            ach = amount / (ns * 1e-9) / 1e9
            peak, unit = HBM, "GB/s"
        else:
            ach = amount / (ns * 1e-9) / 1e12
            peak, unit = BF16, "TFLOP/s"
        table.append({"kernel": key.rstrip("<,"), "calls": cnt, "kernel_ms": ns / 1e6, "share": ns / total_ns,
                      "algorithmic_per_pair": per_pair, "kind": kind, "achieved": ach, "unit": unit, "peak": peak,
                      "frac": ach / peak, "note": note})
    md = ["| kernel | calls | kernel ms | share | achieved | peak | frac | work |", "|---|---|---|---|---|---|---|---|"]
    for t in table:
        md.append("| `%s` | %d | %.1f | %.1f%% | %.0f %s | %.0f | %.3f | %s |" % (
            t["kernel"], t["calls"], t["kernel_ms"], 100 * t["share"], t["achieved"], t["unit"], t["peak"], t["frac"],
            t["note"]))
    print("\n".join(md))
    if a.out:
        with open(a.out + ".json", "w") as f:
            json.dump({"stats": os.path.basename(a.stats), "forwards": a.forwards, "pairs_per_forward": a.pairs,
                       "n": a.n, "table": table}, f, indent=1)
        with open(a.out + ".md", "w") as f:
            f.write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
