"""Per-step interpreter time of the C2 headline from a rocprofv3 kernel trace of
`bench.py --steps S --warmup W --headline-only`, over the timed steps only (the warm-up launches run
while the device is still reaching its clocks): probe + persistent launch durations and the span
from the probe's start to the persistent launch's end -- the interval the bench's HIP events bracket.
Usage: trace_timed_region.py run_kernel_trace.csv STEPS WARMUP [FIRST]
FIRST: the first timed step's launch pair (default WARMUP: the headline's timed steps follow its warm-up
directly; the bench's other step form runs after them)."""
import csv
import statistics as st
import sys

path, steps, warmup = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ek = [r for r in rows if "eval_kernel<float, 16, 2, 0, true>" in r["Kernel_Name"]]
pers = [r for r in ek if r["Grid_Size_X"] == "262144"]
probe = [r for r in ek if r["Grid_Size_X"] != "262144"]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6  # noqa: E731
span = [(int(b["End_Timestamp"]) - int(a["Start_Timestamp"])) / 1e6 for a, b in zip(probe, pers)]
lo = int(sys.argv[4]) if len(sys.argv) > 4 else warmup
lo = max(0, min(lo, len(pers) - steps))
sel = slice(lo, lo + steps)
print(f"launch pairs in the trace: {len(pers)}; timed steps taken: [{lo}, {lo + steps})")
print(f"all launches : persistent {st.mean(map(dur, pers)):.4f} ms, probe {st.mean(map(dur, probe)):.4f} ms, "
      f"probe start -> persistent end {st.mean(span):.4f} ms")
print(f"timed steps  : persistent {st.mean(map(dur, pers[sel])):.4f} ms, probe {st.mean(map(dur, probe[sel])):.4f} ms, "
      f"probe start -> persistent end {st.mean(span[sel]):.4f} ms")
