"""Per-launch-shape durations from a rocprofv3 kernel trace (probe vs persistent launches of the
same kernel symbol differ in grid shape).  python scripts/trace_summary.py run_kernel_trace.csv"""
import collections
import csv
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[(r["Kernel_Name"].split("(")[0][:70], r["Grid_Size_X"], r["Grid_Size_Y"])].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:70s} grid {k[1]:>7s} x {k[2]:>3s}  n={len(v):3d}  avg {sum(v) / len(v):.4f} ms  "
          f"min {min(v):.4f}  max {max(v):.4f}")
