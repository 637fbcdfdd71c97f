"""Per-dispatch PMC counters of the interpreter, split by grid shape (probe vs persistent launch).
    python scripts/pmc_grid.py gpurun_out/abpmc/p1 [kernel-substring]"""
import collections
import csv
import glob
import sys

root = sys.argv[1]
match = sys.argv[2] if len(sys.argv) > 2 else "eval_kernel<float, 16"
for f in sorted(glob.glob(f"{root}/*counter_collection.csv")):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if match not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].split("(")[0], r.get("Grid_Size"), r.get("LDS_Block_Size"))
        d[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in d.items():
        print(k, {n: "%.4g" % (sum(v) / len(v)) for n, v in sorted(c.items())}, "dispatches", len(next(iter(c.values()))))
