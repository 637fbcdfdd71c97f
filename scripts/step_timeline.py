"""Per-step timeline of the C2 bench from a rocprofv3 kernel trace: the dispatches between one
probe launch and the next (kernel, start offset, duration, gap before it), averaged over the steps.
    python scripts/step_timeline.py gpurun_out/trace_c2/.../run_kernel_trace.csv [FIRST COUNT]
FIRST COUNT: the steps to average (default: the last 20)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:60],
       r["Grid_Size_X"], r["Grid_Size_Y"]) for r in rows]
# a step starts at the probe launch (eval_kernel with grid.y > 1 ... the first eval_kernel after a
# reduce): anchor on the persistent launch (the eval_kernel with the largest grid.x) and take the
# dispatch just before it as the probe
big = max(int(e[3]) for e in ev if "eval_kernel" in e[2])
anchors = [i for i, e in enumerate(ev) if "eval_kernel" in e[2] and int(e[3]) == big]
steps = []
for a, b in zip(anchors, anchors[1:]):
    s = a - 1
    steps.append(ev[s:b - 1])
steps = steps[int(sys.argv[2]):int(sys.argv[2]) + int(sys.argv[3])] if len(sys.argv) > 3 else steps[-20:]
prof = collections.defaultdict(lambda: [0.0, 0.0, 0])
for st in steps:
    t0 = st[0][0]
    prev = t0
    for j, (s, e, n, gx, gy) in enumerate(st):
        k = (j, n, gx, gy)
        prof[k][0] += (e - s) / 1e3
        prof[k][1] += (s - prev) / 1e3
        prof[k][2] += 1
        prev = e
tot = sum((st[-1][1] - st[0][0]) / 1e3 for st in steps) / len(steps)
per = sum((steps[i + 1][0][0] - steps[i][0][0]) / 1e3 for i in range(len(steps) - 1)) / (len(steps) - 1)
print(f"steps {len(steps)}: first dispatch start -> last dispatch end {tot:.1f} us; step period {per:.1f} us")
for k, (d, g, c) in sorted(prof.items()):
    print(f"  {k[0]:2d} {k[1]:60s} grid {k[2]:>7s} x {k[3]:>3s}  dur {d / c:8.1f} us  gap before {g / c:7.1f} us")
