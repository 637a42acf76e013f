"""Per-kernel time of one forward from a rocprofv3 kernel trace: the forwards are delimited by the
product-GEMM launches (36 per forward at C3); prints, for the chosen forward, each kernel family's
summed duration, the forward's wall span and the sum of durations (overlap = sum / span).
   python tools/trace_forward.py run_kernel_trace.csv [forward index, default last]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
gem = [i for i, r in enumerate(rows) if "gemm_phase_kernel<0, false>" in r["Kernel_Name"]]
per_fwd = 36
fw = [gem[k:k + per_fwd] for k in range(0, len(gem), per_fwd)]
idx = int(sys.argv[2]) if len(sys.argv) > 2 else len(fw) - 1
lo = fw[idx][0]
hi = fw[idx + 1][0] if idx + 1 < len(fw) else len(rows)
# the forward's first kernels precede its first product GEMM: start from the previous forward's last
# soft top-k / classifier launch + 1 (approximation: 8 launches before the first GEMM)
lo = max(0, lo - 8)
seg = rows[lo:hi]
acc = collections.defaultdict(float)
cnt = collections.Counter()
for r in seg:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name)
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    acc[name] += d
    cnt[name] += 1
span = (max(int(r["End_Timestamp"]) for r in seg) - min(int(r["Start_Timestamp"]) for r in seg)) / 1e6
tot = sum(acc.values())
print("forward %d: %d launches, span %.2f ms, summed kernel time %.2f ms (overlap %.2f)" % (idx, len(seg), span, tot,
                                                                                           tot / span))
for k, v in sorted(acc.items(), key=lambda kv: -kv[1])[:25]:
    print("  %-60s %4d  %7.3f ms  %5.1f%%" % (k[:60], cnt[k], v, 100 * v / tot))
