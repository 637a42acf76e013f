"""Mean PMC counter value per dispatch, grouped by launch position within each repeat block:
   python tools/pmc_dump.py <dir with run_counter_collection.csv> [group]"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
per = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(per)
group = int(sys.argv[2]) if len(sys.argv) > 2 else 23
# gnn_bench: 23 launches per C=17 block (3 warm + 20 timed); phase-split blocks follow
for g0 in range(0, len(ids), group):
    blk = ids[g0 + 3:g0 + group]
    if not blk:
        continue
    keys = sorted(per[blk[0]])
    print("block %d (%d dispatches): " % (g0 // group, len(blk)) +
          "  ".join("%s=%.4g" % (k, sum(per[i][k] for i in blk) / len(blk)) for k in keys))
