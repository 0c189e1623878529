import csv, collections, sys
for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        agg[r['Kernel_Name']][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, d in agg.items():
        if 'rocclr' in k: continue
        print(k.split('(')[0][:28], " ".join(f"{c}={sum(v)/len(v):.3e}" for c, v in sorted(d.items())))
