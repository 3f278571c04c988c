"""Timeline of one training step from a rocprofv3 kernel_trace.csv: every kernel of the last
complete step (a step starts at each launch of the marker kernel, default k_prep_pass1_q) with
its start offset, duration, queue, the gap the device sat idle before it, and the step's span,
busy union and idle total.  usage: step_timeline.py <kernel_trace.csv> [marker] [step index]"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "k_prep_pass1_q"
rows = []
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r.get("Queue_Id", "?"),
                 r.get("Grid_Size_X", r.get("Grid_Size", "?"))))
rows.sort()
starts = [i for i, r in enumerate(rows) if r[2].startswith(marker)]
if len(starts) < 2:
    sys.exit(f"fewer than two '{marker}' launches in the trace")
k = int(sys.argv[3]) if len(sys.argv) > 3 else len(starts) - 2
step = rows[starts[k]:starts[k + 1]]
t0 = step[0][0]
busy_end = t0
busy = idle = 0
print(f"step {k} of {len(starts) - 1}: {len(step)} kernels")
print(f"{'start':>8s} {'dur':>7s} {'gap':>6s}  q   kernel (grid)")
for s, e, n, q, gx in step:
    gap = max(0, s - busy_end)
    idle += gap
    if e > busy_end:
        busy += e - max(s, busy_end)
        busy_end = e
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {gap / 1e3:6.1f}  {q:>2s}  {n[:48]} ({gx})")
span = (step[-1][1] if step[-1][1] > busy_end else busy_end) - t0
print(f"span {span / 1e3:.1f} us (to the last end), busy union {busy / 1e3:.1f} us, idle gaps {idle / 1e3:.1f} us; "
      f"next step starts at {(rows[starts[k + 1]][0] - t0) / 1e3:.1f} us")
