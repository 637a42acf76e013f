"""Per-kernel PMC summary of a tools/pmc_kernel.sh output directory:
   python tools/pmc_table.py gpurun_out/pmc_r02 [out.json]
Means per dispatch for every counter of every pass, grouped by kernel name (template args kept up
to the first '('), plus derived ratios:
  valu_busy  = SQ_ACTIVE_INST_VALU / (SQ_WAVE_CYCLES / waves-resident) -- VALU issue share
  wait_ratio = SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY
  hbm_bytes  = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B; gfx950 FETCH_SIZE reports half the bytes of
               16-B/lane reads, MI355X_MICROARCH.md HBM section)
  l2_hit     = TCC_HIT / (TCC_HIT + TCC_MISS)"""
import csv
import json
import os
import sys
from collections import defaultdict

src = sys.argv[1]
acc = defaultdict(lambda: defaultdict(dict))   # kernel -> counter -> dispatch -> value
for p in sorted(os.listdir(src)):
    f = os.path.join(src, p, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "", 1).split("(")[0]
        d = acc[k][r["Counter_Name"]]
        d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])

out = {}
for k, cs in sorted(acc.items()):
    m = {c: sum(v.values()) / len(v) for c, v in cs.items()}
    m["dispatches"] = max(len(v) for v in cs.values())
    g = lambda c: m.get(c)
    if g("SQ_WAIT_INST_ANY") and g("SQ_ACTIVE_INST_ANY"):
        m["wait_ratio"] = g("SQ_WAIT_INST_ANY") / g("SQ_ACTIVE_INST_ANY")
    if g("SQ_ACTIVE_INST_VALU") and g("SQ_ACTIVE_INST_ANY"):
        m["valu_share_of_active"] = g("SQ_ACTIVE_INST_VALU") / g("SQ_ACTIVE_INST_ANY")
    if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
        m["valu_insts_per_wave"] = g("SQ_INSTS_VALU") / g("SQ_WAVES")
    if g("SQ_INSTS_LDS") and g("SQ_WAVES"):
        m["lds_insts_per_wave"] = g("SQ_INSTS_LDS") / g("SQ_WAVES")
    if g("SQ_LDS_BANK_CONFLICT") is not None and g("SQ_ACTIVE_INST_LDS"):
        m["lds_conflict_per_active"] = g("SQ_LDS_BANK_CONFLICT") / g("SQ_ACTIVE_INST_LDS")
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        m["hbm_bytes"] = (2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024
    if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum"):
        m["l2_hit"] = g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))
    out[k] = m

keys = ["dispatches", "SQ_WAVES", "SQ_BUSY_CYCLES", "valu_insts_per_wave", "lds_insts_per_wave", "wait_ratio",
        "valu_share_of_active", "lds_conflict_per_active", "hbm_bytes", "l2_hit"]
print("%-44s " % "kernel" + " ".join("%12s" % c[:12] for c in keys))
for k, m in out.items():
    print("%-44s " % k[:44] + " ".join("%12.4g" % m[c] if c in m else "%12s" % "-" for c in keys))
if len(sys.argv) > 2:
    json.dump({"source": src, "kernels": out}, open(sys.argv[2], "w"), indent=1)
