"""Where a C4 optimize_constants call spends the device (rocprofv3 kernel trace of `bench.py --config c4`).
    python scripts/c4_trace.py run_kernel_trace.csv [--json out.json]
Takes the last optimize_constants call in the trace (from the interpreter launch of its baseline
evaluation to that of its final one), then reports: wall span, device-busy time (union of kernel intervals over all queues),
kernel time by kernel name and by grid-size class, and the idle gaps (count and sum) between
consecutive kernels of each queue."""
import collections
import csv
import json
import re
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    ev = []
    for r in rows:
        ev.append(dict(s=int(r["Start_Timestamp"]), e=int(r["End_Timestamp"]),
                       name=r["Kernel_Name"].split("(")[0], gx=int(r["Grid_Size_X"]),
                       q=r.get("Queue_Id", r.get("Stream_Id", "0"))))
    ev.sort(key=lambda x: x["s"])
    return ev


def last_call(ev):
    # every optimize_constants call starts and ends with an evaluation of the population by the
    # interpreter (the baseline losses, the returned trees' losses): the last call is the span from the
    # second-to-last interpreter launch over the whole population to the last one
    big = [i for i, x in enumerate(ev) if re.search(r"eval_kernel<double, \d+, \d+, 0,", x["name"])]
    if len(big) < 2:
        return ev
    return ev[big[-2]:big[-1] + 1]


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def size_class(gx):
    w = gx // 64
    for lim in (64, 512, 4096, 32768):
        if w <= lim:
            return f"<= {lim} waves"
    return "> 32768 waves"


def main():
    ev = last_call(load(sys.argv[1]))
    span = (ev[-1]["e"] - ev[0]["s"]) / 1e6
    busy = union([(x["s"], x["e"]) for x in ev]) / 1e6
    by_name = collections.defaultdict(lambda: [0, 0.0])
    by_cls = collections.defaultdict(lambda: [0, 0.0])
    for x in ev:
        d = (x["e"] - x["s"]) / 1e6
        short = x["name"].replace("srhip::", "")[:60]
        by_name[short][0] += 1
        by_name[short][1] += d
        if "grad_kernel" in x["name"]:
            k = size_class(x["gx"])
            by_cls[k][0] += 1
            by_cls[k][1] += d
    gaps = collections.defaultdict(lambda: [0, 0.0])
    byq = collections.defaultdict(list)
    for x in ev:
        byq[x["q"]].append(x)
    for q, xs in byq.items():
        for a, b in zip(xs, xs[1:]):
            g = (b["s"] - a["e"]) / 1e6
            if g > 0:
                gaps[q][0] += 1
                gaps[q][1] += g
    hist = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
    for x in ev:
        if "grad_kernel" in x["name"] and "reduce" not in x["name"]:
            d = (x["e"] - x["s"]) / 1e3
            b = next((f"<= {lim} us" for lim in (10, 20, 40, 80, 160, 320, 640) if d <= lim), "> 640 us")
            h = hist[x["name"].split("<")[1].split(",")[1].strip() + "-wide"]
            h[b][0] += 1
            h[b][1] += d / 1e3
    out = {"span_ms": span, "busy_ms": busy, "kernels": len(ev),
           "by_kernel": {k: {"n": v[0], "ms": v[1], "us_each": 1e3 * v[1] / v[0]} for k, v in
                         sorted(by_name.items(), key=lambda kv: -kv[1][1])},
           "grad_by_grid": {k: {"n": v[0], "ms": v[1], "us_each": 1e3 * v[1] / v[0]} for k, v in sorted(by_cls.items())},
           "grad_duration_hist": {k: {b: {"n": v[0], "ms": v[1]} for b, v in sorted(h.items())} for k, h in hist.items()},
           "queue_gaps": {q: {"n": v[0], "ms": v[1]} for q, v in gaps.items()},
           "launches_per_queue": {q: len(xs) for q, xs in byq.items()}}
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
