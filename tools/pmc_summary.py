"""Average PMC counter values per kernel over rocprofv3 counter_collection CSVs.
usage: python tools/pmc_summary.py gpurun_out/<tag>/p*/run_counter_collection.csv"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "rocclr" in k:
        continue
    print(k[:40])
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v) / len(v):.4e}")
