"""Timeline of the last timed forward from a rocprofv3 kernel_trace.csv: kernels that end after the
last soft top-k (the critical-path tail behind the GPU stage).  python tools/tail_trace.py CSV"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
topk = [r for r in rows if "soft_topk_kernel" in r["Kernel_Name"]]
# forward boundaries: GPU-idle gaps > 1 ms split the trace into segments; take the last segment
# holding a full forward (>= 8 soft top-k launches) before the bench's isolated single-stream run
segs, cur = [], None
for r in rows:
    if cur is None or r["s"] - cur[1] > 1_000_000:
        cur = [r["s"], r["e"], []]
        segs.append(cur)
    cur[1] = max(cur[1], r["e"])
    cur[2].append(r)
full = [sg for sg in segs if sum("soft_topk_kernel" in r["Kernel_Name"] for r in sg[2]) >= 8]
for sg in full:
    print("segment %.2f ms, %d kernels" % ((sg[1] - sg[0]) / 1e6, len(sg[2])))
sg = full[-2] if len(full) > 2 else full[-1]
t0 = sg[0]
fw = sg[2]
last_topk = max(r["e"] for r in fw if "soft_topk_kernel" in r["Kernel_Name"])
end = max(r["e"] for r in fw)
print("forward span %.2f ms, last soft_topk at %.2f ms, last kernel %.2f ms" % ((end - t0) / 1e6, (last_topk - t0) / 1e6,
                                                                                 (end - t0) / 1e6))
agg = {}
for r in fw:
    if r["e"] > last_topk:
        k = r["Kernel_Name"][:60]
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += (r["e"] - max(r["s"], last_topk)) / 1e6
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%-60s %4d %7.3f ms" % (k, c, t))
busy = sorted((r["s"], r["e"]) for r in fw)
gaps, cur = 0, t0
for s, e in busy:
    if s > cur:
        gaps += s - cur
    cur = max(cur, e)
print("idle time inside the forward: %.2f ms" % (gaps / 1e6))
