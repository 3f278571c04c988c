"""Average PMC counter values per kernel from a rocprofv3 counter_collection CSV."""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r['Kernel_Name'].split('(')[0][-40:]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in agg.items():
    if 'rocclr' in k or 'at::native' in k:
        continue
    print(f"{k:40s}", {c: f"{sum(v) / len(v):.4g}" for c, v in d.items()})
