"""Per-STEP counter totals of a kernel symbol from rocprofv3 --pmc passes (the persistent C2 step
launches the interpreter twice -- probe + persistent launch -- under one symbol): sums every
dispatch of the kernel and divides by the step count.  HBM bytes per MI355X_MICROARCH.md (gfx950):
fetch = 2 x 1024 x FETCH_SIZE, write = 1024 x WRITE_SIZE (KiB counters).
    python scripts/pmc_step.py ROOT STEPS [kernel-substring] [--json out.json]"""
import collections
import csv
import glob
import json
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
if out_json in args:
    args.remove(out_json)
root, steps = args[0], int(args[1])
match = args[2] if len(args) > 2 else "eval_kernel<float, 16, 2, 0, true>"
# a counter collected in several passes (GRBM_GUI_ACTIVE rides along in each) is averaged over them
tot = collections.defaultdict(lambda: collections.defaultdict(float))
npass = collections.defaultdict(lambda: collections.defaultdict(set))
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("void ", "")
        if match not in k:
            continue
        tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
        npass[k][row["Counter_Name"]].add(f)
summary = {}
for k, c in tot.items():
    per = {n: v / steps / len(npass[k][n]) for n, v in c.items()}
    d = {"counters_per_step": per, "steps": steps}
    if "FETCH_SIZE" in per:
        d["hbm_fetch_bytes"] = 2 * 1024 * per["FETCH_SIZE"]
    if "WRITE_SIZE" in per:
        d["hbm_write_bytes"] = 1024 * per["WRITE_SIZE"]
    if "hbm_fetch_bytes" in d and "hbm_write_bytes" in d:
        d["hbm_bytes"] = d["hbm_fetch_bytes"] + d["hbm_write_bytes"]
    if "SQ_ACTIVE_INST_VALU" in per and "GRBM_GUI_ACTIVE" in per:
        # GRBM_GUI_ACTIVE sums the 8 XCDs' cycles; one VALU issue slot per SIMD per 4 cycles... as
        # the round-2 summaries: ACTIVE_INST_VALU x 4 / (GUI cycles per XCD x 1024 SIMDs)
        d["valu_issue_util"] = per["SQ_ACTIVE_INST_VALU"] * 4 / (per["GRBM_GUI_ACTIVE"] / 8 * 1024)
    summary[k] = d
print(json.dumps(summary, indent=1))
if out_json:
    json.dump(summary, open(out_json, "w"), indent=1)
