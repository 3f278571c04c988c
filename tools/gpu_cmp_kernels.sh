#!/bin/bash
# two kernel traces of the ratio forward (in-tree vs $1) and a per-kernel comparison
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/${TAG:-pr}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o run -- python3 tools/prof_ratio.py > $O/new.log 2>&1 || { tail $O/new.log; exit 1; }
RGBD_HIP_LIB=$GRAFT_REPO_ROOT/$1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o run -- python3 tools/prof_ratio.py > $O/old.log 2>&1 || { tail $O/old.log; exit 1; }
find $O -name "*kernel_stats.csv" | sort
python3 - "$O" <<'PY'
import csv, sys
O = sys.argv[1]
def load(p):
    return {r['Name'][:60]: (int(r['Calls']), float(r['AverageNs']) / 1000, float(r['TotalDurationNs']) / 1000)
            for r in csv.DictReader(open(p))}
n, o = load(f"{O}/new/run_kernel_stats.csv"), load(f"{O}/old/run_kernel_stats.csv")
z = (0, 0.0, 0.0)
for k in sorted(set(n) | set(o), key=lambda k: -max(n.get(k, z)[2], o.get(k, z)[2])):
    a, b = n.get(k, z), o.get(k, z)
    print(f"{k:60s} new {a[0]:4d} x {a[1]:8.1f}   old {b[0]:4d} x {b[1]:8.1f}")
print("sum of averages x calls / iters: new", round(sum(v[2] for v in n.values()) / 30, 1), "old", round(sum(v[2] for v in o.values()) / 30, 1))
PY
