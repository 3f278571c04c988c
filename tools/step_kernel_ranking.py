"""Per-kernel time of ONE steady-state training step from a rocprofv3 kernel_trace.csv, ranked:
the step is the interval between the last two launches of the marker kernel (default
k_prep_pass1_q, the first kernel of every step: K1's assembly), so warm-up work (MIOpen's
solver search, first-call packing) is excluded.  Groups kernels by a short family name.
usage: step_kernel_ranking.py <kernel_trace.csv> [marker] [top]"""
import collections
import csv
import re
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_prep_pass1_q"
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = []
for r in csv.DictReader(open(path)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
starts = [i for i, r in enumerate(rows) if marker in r[2]]
if len(starts) < 2:
    sys.exit(f"fewer than two '{marker}' launches")
step = rows[starts[-2]:starts[-1]]
span = (step[-1][1] - step[0][0]) / 1e3
busy = collections.Counter()
calls = collections.Counter()


def family(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"^rgbd::", "", n)
    if n.startswith("Cijk_"):
        return "hipBLASLt/Tensile GEMM " + n.split("_MT")[1].split("_")[0] if "_MT" in n else "Tensile GEMM"
    if n.startswith("_ZN2ck"):
        return "CK " + re.sub(r"\d+", "", n[6:60])
    return n.split("(")[0][:90]


for s, e, n in step:
    f = family(n)
    busy[f] += (e - s) / 1e3
    calls[f] += 1
tot = sum(busy.values())
print(f"step span {span:.1f} us, kernel time {tot:.1f} us, {len(step)} launches")
for f, t in busy.most_common(top):
    print(f"{t:10.1f} us {100 * t / tot:5.1f}% {calls[f]:5d}  {f}")
