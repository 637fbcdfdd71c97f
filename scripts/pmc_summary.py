"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/...counter_collection.csv) per kernel."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
match = sys.argv[2] if len(sys.argv) > 2 else "eval_kernel"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/p*/p*_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if match not in k:
            continue
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        cnt[k][row["Counter_Name"]] += 1
for k, v in agg.items():
    print(k)
    for c, x in sorted(v.items()):
        print(f"  {c:28s} {x / cnt[k][c]:.4g}")
