"""Per (kernel, grid) average duration from a rocprofv3 kernel_trace CSV: python tools/trace_shapes.py CSV [substr ...]"""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
pats = sys.argv[2:]
d = collections.defaultdict(list)
order = []
for r in rows:
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0]
    if pats and not any(p in n for p in pats):
        continue
    key = (n[-32:], f"{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}", r['Workgroup_Size_X'])
    if key not in d:
        order.append(key)
    d[key].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
for k in order:
    v = d[k]
    print(f"{k[0]:34s} grid {k[1]:>18s} wg {k[2]:>4s}  n={len(v):3d}  avg {sum(v) / len(v) / 1e3:8.1f} us")
