"""From a rocprofv3 kernel trace: per queue, do consecutive kernels overlap? and the mean
duration per kernel name.  usage: python tools/stream_overlap.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
byq = collections.defaultdict(list)
dur = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].split("(")[0]
    if not name.startswith("jit_"):
        continue
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    byq[(r.get("Queue_Id"), r.get("Stream_Id"))].append((s, e, name))
    dur[name].append((e - s) / 1e3)
for q, ks in byq.items():
    ks.sort()
    ov = [(a[2], b[2], (a[1] - b[0]) / 1e3) for a, b in zip(ks, ks[1:]) if b[0] < a[1]]
    print("queue/stream", q, "kernels", len(ks), "overlapping successors", len(ov), ov[:6])
for n, d in dur.items():
    print(n, "mean us", round(sum(d) / len(d), 2), "n", len(d))
