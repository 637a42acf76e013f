"""Summarise a rocprofv3 kernel_stats.csv per forward: python tools/kstats.py CSV NFWD [TOP]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nf = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(r['TotalDurationNs']) for r in rows)
print('total ms per forward %.2f' % (tot / nf / 1e6))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:top]:
    print("%-64s %5s %8.3f ms/fwd  avg %7.3f ms %5.1f%%" % (r['Name'][:64], r['Calls'], float(r['TotalDurationNs']) / nf / 1e6,
                                                            float(r['AverageNs']) / 1e6, 100 * float(r['TotalDurationNs']) / tot))
