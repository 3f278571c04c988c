"""Average duration per (kernel, grid) from a rocprofv3 kernel_trace.csv; optional name filter."""
import collections, csv, sys
d = collections.defaultdict(list)
meta = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0]
    if len(sys.argv) > 2 and sys.argv[2] not in n:
        continue
    k = (n, r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])
    d[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
    meta[k] = (r['VGPR_Count'], r['Accum_VGPR_Count'], r['LDS_Block_Size'])
for k, v in d.items():
    print(f"{k[0][:40]:40s} grid {k[1]:>8s} {k[2]:>4s} {k[3]:>4s}  n={len(v):3d}  avg {sum(v)/len(v):8.1f} us  vgpr/agpr/lds {meta[k]}")
