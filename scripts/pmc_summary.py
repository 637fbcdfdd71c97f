"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/...counter_collection.csv) per kernel.

    python scripts/pmc_summary.py [root] [kernel-substring] [--json out.json]

Counters are averaged per dispatch class: when one kernel symbol has dispatches of very different
durations (the C2 probe and persistent launches share a symbol, grid size and static LDS), the
dispatches above the geometric mean of the shortest and longest keep the plain kernel name and the
others are summarised apart as "<name> [short]".  HBM bytes follow MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE
and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide coalesced read, so
fetch bytes = 2 x 1024 x FETCH_SIZE and write bytes = 1024 x WRITE_SIZE.
"""
import collections
import csv
import glob
import json
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
if out_json in args:
    args.remove(out_json)
root = args[0] if len(args) > 0 else "gpurun_out/pmc"
match = args[1] if len(args) > 1 else "eval_kernel"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
rows = collections.defaultdict(list)  # kernel -> [(pass file, dispatch id, counter, value, duration)]
for f in sorted(glob.glob(f"{root}/p*/p*_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if match not in row["Kernel_Name"]:
            continue
        rows[row["Kernel_Name"]].append((f, row["Dispatch_Id"], row["Counter_Name"], float(row["Counter_Value"]),
                                         int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
for k, rs in rows.items():
    lo, hi = min(r[4] for r in rs), max(r[4] for r in rs)
    cut = (lo * hi) ** 0.5 if hi > 3 * lo else -1
    for f, did, name, val, d in rs:
        key = k if d >= cut else f"{k} [short]"
        agg[key][name] += val
        cnt[key][name] += 1
summary = {}
for k, v in agg.items():
    c = {name: x / cnt[k][name] for name, x in v.items()}
    d = {"counters_per_dispatch": c}
    if "FETCH_SIZE" in c:
        d["hbm_fetch_bytes"] = 2 * 1024 * c["FETCH_SIZE"]
    if "WRITE_SIZE" in c:
        d["hbm_write_bytes"] = 1024 * c["WRITE_SIZE"]
    if "hbm_fetch_bytes" in d and "hbm_write_bytes" in d:
        d["hbm_bytes"] = d["hbm_fetch_bytes"] + d["hbm_write_bytes"]
    if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c:
        # VALU issue utilisation: one wave64 VALU instruction occupies a SIMD for 4 cycles;
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs
        d["valu_issue_util"] = c["SQ_INSTS_VALU"] * 4 / 1024 / (c["GRBM_GUI_ACTIVE"] / 8)
    summary[k] = d
    print(k)
    for name, x in sorted(c.items()):
        print(f"  {name:28s} {x:.4g}")
    for key in ("hbm_fetch_bytes", "hbm_write_bytes", "hbm_bytes", "valu_issue_util"):
        if key in d:
            print(f"  {key:28s} {d[key]:.4g}")
if out_json:
    json.dump(summary, open(out_json, "w"), indent=1, sort_keys=True)
