"""The coalescer under native client threads (tools/coalescer_bench.cpp, no Python GIL in the
request path): writes a tree pool and dataset, runs the driver for each client count, prints its
JSON lines.  python scripts/coalescer_native.py [c1|c3] [clients ...]
  c1: the README example's shape, 2 features x 100 rows Float64, + * / - cos exp;
  c3: 10 features x 100k rows Float32 (a C3-shape row subset)."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

import numpy as np  # noqa: E402

import srhip  # noqa: E402
from srhip import _lib  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "c1"
clients = [int(c) for c in sys.argv[2:]] or [1, 4, 16, 64]
opts = srhip.Options(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))
if shape == "c1":
    dtype, nfeat, n = np.float64, 2, 100
else:
    dtype, nfeat, n = np.float32, 10, 100_000
rng = np.random.default_rng(0)
X = rng.standard_normal((nfeat, n)).astype(dtype)
y = (2 * np.cos(X[1]) + X[0] ** 2 - 2).astype(dtype)
trees = srhip.random_population(2048, opts, nfeat, dtype, seed=1, max_size=20)
nodes, offs = srhip.flatten(trees, opts, dtype)
d = tempfile.mkdtemp(prefix="coalescer_")
nodes.tofile(os.path.join(d, "nodes.bin"))
np.asarray(offs, dtype=np.int64).tofile(os.path.join(d, "offs.bin"))
X.tofile(os.path.join(d, "X.bin"))
y.tofile(os.path.join(d, "y.bin"))
with open(os.path.join(d, "meta.txt"), "w") as f:
    f.write(f"{_lib.dtype_code(dtype)} {nfeat} {n} {len(offs) - 1} {len(opts.binop_codes)} {len(opts.unaop_codes)}\n")
    f.write(" ".join(str(int(c)) for c in opts.binop_codes) + "\n")
    f.write(" ".join(str(int(c)) for c in opts.unaop_codes) + "\n")
exe = os.path.join(ROOT, "tools", "build", "coalescer_bench")
for c in clients:
    out = subprocess.run([exe, d, str(c), os.environ.get("SECONDS_PER_RUN", "3")], capture_output=True, text=True,
                         timeout=120)
    if out.returncode != 0:
        print(out.stderr, file=sys.stderr)
        sys.exit(out.returncode)
    if os.environ.get("SRHIP_HOST_TIMING"):
        print(out.stderr, file=sys.stderr)
    line = json.loads(out.stdout.strip().splitlines()[-1])
    line["shape"] = shape
    print(json.dumps(line), flush=True)
