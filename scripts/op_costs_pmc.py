"""Counters per operator from rocprofv3 --pmc passes over scripts/op_costs.py: each eval's
eval_kernel dispatches (those before its reduce_kernel) are summed and attributed to the shape
gpurun_out/op_costs_order.json lists at that position; the last repetition of a shape is kept.
Per shape: counters per launch and, against the leaf baseline, wave-instructions x 64 lanes per
operator-node-row.  python scripts/op_costs_pmc.py PMC_ROOT ORDER_JSON [--json out.json]"""
import collections
import csv
import glob
import json
import re
import sys

root, order_path = sys.argv[1], sys.argv[2]
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
meta = json.load(open(order_path))
order, shapes = meta["order"], meta["shapes"]
per_shape = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    disp = collections.defaultdict(dict)
    names = {}
    for row in csv.DictReader(open(f)):
        d = int(row["Dispatch_Id"])
        names[d] = row["Kernel_Name"]
        disp[d][row["Counter_Name"]] = disp[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    ev, acc = 0, collections.defaultdict(float)
    for d in sorted(disp):
        m = re.search(r"eval_kernel<\w+, \d+, \d+, (\d+)", names[d])
        if m and m.group(1) != "2":  # the interpreter's loss launches (MODE 2: the precise pass, after the reduction)
            for k, v in disp[d].items():
                acc[k] += v
        elif re.search(r"(^|[^_])reduce_kernel<", names[d]) and acc:  # the loss reduction (not precise_reduce_kernel)
            if ev < len(order):
                per_shape[order[ev]].update(acc)  # later repetitions overwrite earlier ones
            ev += 1
            acc = collections.defaultdict(float)
rows = 1_000_000
base = per_shape.get("leaf", {})
out = {}
for name, c in per_shape.items():
    s = shapes[name]
    d = {"counters": dict(c), "opnodes": s["opnodes"], "kernel_ms": s["kernel_ms"]}
    if name != "leaf" and base and s["opnodes"]:
        d["lane_instr_per_opnode_row"] = {k: (c[k] - base.get(k, 0.0)) * 64 / (s["opnodes"] * rows)
                                          for k in c if k.startswith("SQ_INSTS")}
        d["wave_instr_per_opnode_tile"] = {k: (c[k] - base.get(k, 0.0)) / (s["opnodes"] * rows / 1024)
                                           for k in c if k.startswith("SQ_INSTS")}
        d["ns_per_opnode_row_x1e3"] = (s["kernel_ms"] - shapes["leaf"]["kernel_ms"]) * 1e9 / (s["opnodes"] * rows)
    out[name] = d
print(json.dumps(out, indent=1))
if out_json:
    json.dump(out, open(out_json, "w"), indent=1)
