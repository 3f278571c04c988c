"""Average PMC counter values per (kernel, grid) from rocprofv3 counter_collection CSVs."""
import collections, csv, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
order = []
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')
        if 'rocclr' in n or 'at::native' in n:
            continue
        key = (n[-28:], r['Grid_Size'])
        if key not in agg:
            order.append(key)
        agg[key][r['Counter_Name']].append(float(r['Counter_Value']))
for k in order:
    d = agg[k]
    print(f"{k[0]:28s} {k[1]:>9s}", " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in d.items()))
