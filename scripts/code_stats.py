"""Instruction-mix study of a compiled population (diagnostic): handler frequencies, adjacent pairs,
instructions per tree, for the C2 bench population.  Uses SRHIP_DUMP_CODE (host compile only)."""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "symbolicregression.jl_amd"))
os.environ["SRHIP_DUMP_CODE"] = "/tmp/srhip_code.bin"
import srhip as sr  # noqa: E402
from srhip import workloads  # noqa: E402

opts, X, y, trees, nodes, offs = workloads.c2(0, 1024, 4096)
sr.Program(None, nodes, offs, opts, np.float32)
rec = np.fromfile("/tmp/srhip_code.bin", dtype=np.int32).reshape(-1, 4)[:, :2]

# handler names (srhip_isa.h layout)
K_MAX = 8
SB = ["ADD", "SUB", "MUL", "DIV", "GT", "COND", "OR", "AND", "MAX", "MIN"]
UN = ["NEG", "SQUARE", "CUBE", "ABS", "RELU", "COS", "SIN", "TAN", "EXP", "LOG"]
H_SLOADF0, H_SLOADC0, H_PUSH0 = 3, 3 + K_MAX, 3 + 2 * K_MAX
H_PUSHLF0, H_PUSHLC0 = H_PUSH0 + K_MAX, H_PUSH0 + 2 * K_MAX
H_BIN0 = H_PUSHLC0 + K_MAX
SPEC_STRIDE = 4 + 2 * K_MAX + 3
FORMS = ["AF", "FA", "AC", "CA"] + [f"SA{k}" for k in range(K_MAX)] + [f"AS{k}" for k in range(K_MAX)] + ["FF", "FC", "CF"]
H_HEAVY0 = H_BIN0 + 10 * SPEC_STRIDE
H_UN0 = H_HEAVY0 + 3 * 2 * K_MAX
NUN = 33


def name(h):
    if h == 0: return "END"
    if h == 1: return "LOADF"
    if h == 2: return "LOADC"
    if h < H_SLOADC0: return f"SLOADF{h - H_SLOADF0}"
    if h < H_PUSH0: return f"SLOADC{h - H_SLOADC0}"
    if h < H_PUSHLF0: return f"PUSH{h - H_PUSH0}"
    if h < H_PUSHLC0: return f"PUSHLF{h - H_PUSHLF0}"
    if h < H_BIN0: return f"PUSHLC{h - H_PUSHLC0}"
    if h < H_HEAVY0:
        sb, f = divmod(h - H_BIN0, SPEC_STRIDE)
        form = FORMS[f]
        return f"{SB[sb]}_{form}"
    if h < H_UN0: return f"HEAVY{h - H_HEAVY0}"
    if h < H_UN0 + NUN:
        u = h - H_UN0
        return f"UN_{UN[u] if u < len(UN) else u}"
    return {H_UN0 + NUN: "COS_NC", H_UN0 + NUN + 1: "SIN_NC"}.get(h, f"h{h}")


hs, pairs, lens, cur, fails = collections.Counter(), collections.Counter(), [], [], 0
for h, a in rec:
    if h == -1:
        lens.append(len(cur))
        fails += a
        for u, v in zip(cur, cur[1:]):
            pairs[(u, v)] += 1
        cur = []
        continue
    nm = name(int(h))
    hs[nm] += 1
    cur.append(nm)
tot = sum(hs.values())
print(f"trees {len(lens)} (static fail {fails}), instructions {tot}, per tree {tot / len(lens):.2f}, max {max(lens)}")
for nm, c in hs.most_common(40):
    print(f"  {nm:12s} {c:6d} {100 * c / tot:5.1f}%")
print("top adjacent pairs:")
for (u, v), c in pairs.most_common(25):
    print(f"  {u:10s} -> {v:10s} {c:6d} {100 * c / tot:5.1f}%")
