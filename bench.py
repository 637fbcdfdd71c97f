"""bench.py — BASELINE.json's headline metric on config C2:
1024 random trees (size U{1..30}, ops + - * / cos exp) x 1M rows x 5 features, Float32, fused L2
loss, one MI355X per rank.  A step = one srhip_eval_loss over the whole population (dataset
and compiled population resident in HBM; per-step host work: launch, per-tree did_succeed
decisions, 1024 losses back to the host).  `value` counts the node-rows the device actually
evaluated (srhip_last_work: a failed tree's skipped rows are not counted).  Steps are issued as
the search issues populations: step k + 1 submitted (srhip_eval_loss_submit) before step k is
waited for; --sync times blocking srhip_eval_loss calls instead (both forms are in the line).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cpu-seconds S] [--mode islands|rowshard]

N > 1 (launched by torch.distributed.run), --mode islands (default): each rank evaluates its own
population on its own GPU (islands, src/SymbolicRegression.jl:746-793) and every step's results
feed the migration exchange (src/Migration.jl:16-38): each rank's 12 best trees reach every rank
through one RCCL all_gather_into_tensor, in flight during the next step's evaluation; weak
scaling.  --mode rowshard: one population over a 10 x 10M dataset whose rows are sharded over the
ranks, one fused all-reduce of the per-tree partials per step; strong scaling.  Barrier +
max-over-ranks timing via torch.distributed.  --config c4 / c1 / c3: the other BASELINE configs.
Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "symbolicregression.jl_amd"))

PEAK_FP32_TFLOPS = 157.3  # MI355X FP32 vector (= FP32 MFMA) peak, MI355X_MICROARCH.md
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 vector peak


class _Done:
    """A synchronous evaluation's result in the shape of an EvalTicket (the timed loops take either)."""

    def __init__(self, res):
        self.res = res

    def wait(self):
        return self.res


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE when launched by torch.distributed.run, else 1). "
                         "Without WORLD_SIZE and N > 1 the bench starts the N ranks itself (torch.distributed.run "
                         "child, before any GPU call) and exits with the worst rank's status")
    ap.add_argument("--launch-check", action="store_true",
                    help="(tests) every rank prints its rank / world / device assignment as JSON and exits before "
                         "touching the GPU")
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default: c2 20, c4 10)")
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed steps first (default: c2 30 -- the GPU reaches its steady clocks over the "
                         "first ~50 ms of work -- c4 3)")
    ap.add_argument("--ntrees", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--headline-only", action="store_true",
                    help="c2: skip the extra lines (derived columns, no early exit) -- profiler runs, whose "
                         "per-kernel average must be the headline kernel's alone")
    ap.add_argument("--binops", default="+,-,*,/", help="(tuning) binary operators of the C2 population")
    ap.add_argument("--unaops", default="cos,exp", help="(tuning) unary operators of the C2 population")
    ap.add_argument("--mode", default="islands", choices=("islands", "rowshard"),
                    help="c2 over N ranks: islands (each rank its own population; every step ends with the "
                         "migration all-gather of each rank's best trees) or rowshard (one population, the "
                         "C3-shape 10 x 10M dataset's rows sharded over the ranks, one all-reduce of the "
                         "per-tree partials per step: strong scaling)")
    ap.add_argument("--sync", action="store_true",
                    help="c2: time one synchronous srhip_eval_loss per step instead of the submit/wait "
                         "pipeline (both are reported; this picks the headline)")
    ap.add_argument("--depth", type=int, default=2, help="c2: evaluations in flight in the pipelined step (2-3)")
    ap.add_argument("--migrate-k", type=int, default=12, help="islands: trees each rank sends per step (topn)")
    ap.add_argument("--config", default="c2", choices=("c2", "c4", "c1", "c3"),
                    help="c2 (default, the headline metric); c4: batched constant optimisation; c1 / c3: "
                         "equation_search (README example / 10M x 10 islands over the ranks)")
    ap.add_argument("--iterations", type=int, default=0,
                    help="c1/c3: search iterations (default: c1 2 of the config's 40, c3 1)")
    ap.add_argument("--ncycles", type=int, default=0, help="c1/c3: ncycles_per_iteration (default 550)")
    ap.add_argument("--parallelism", default="multithreading", choices=("multithreading", "multiprocessing"),
                    help="c1/c3: islands as threads of one process, or in worker processes (:multiprocessing)")
    ap.add_argument("--procs", type=int, default=0, help="c1/c3 multiprocessing: worker processes "
                    "(default min(populations per GPU, 16))")
    args = ap.parse_args(argv)
    if args.steps is None:
        args.steps = 20 if args.config == "c2" else 10
    if args.warmup is None:
        args.warmup = 30 if args.config == "c2" else 3
    return args


def rank_plan(gpus, env):
    """How this process runs `--gpus gpus` given its environment: ("launch", N) when it must start N ranks
    itself (no WORLD_SIZE, N > 1), ("run", N) when it is one of N ranks (or the only one).  A WORLD_SIZE
    that disagrees with an explicit --gpus is an error: the line would report a rank count it did not
    run."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        n = 1 if gpus is None else int(gpus)
        if n < 1:
            raise SystemExit(f"bench.py: --gpus {n} < 1")
        return ("launch", n) if n > 1 else ("run", 1)
    ws = int(ws)
    if gpus is not None and int(gpus) != ws:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws} (launched with a different rank count)")
    return "run", ws


def free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_cmd(n, argv, port):
    """The child command that runs this bench as n ranks on one node (the driver's own form)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """Start the n ranks as ONE child process (torch.distributed.run) -- this process has made no GPU or
    torch call, so nothing is inherited or exec'd over an initialised runtime -- and return the child's
    status (torch.distributed.run fails when any rank fails).  Rank 0 prints the JSON line."""
    import subprocess

    return subprocess.call(launch_cmd(n, argv, free_port()))


def main():
    args = parse()
    plan, n = rank_plan(args.gpus, os.environ)
    if plan == "launch":  # (an explicit --gpus N > 1 is in argv: every rank re-reads it)
        sys.exit(launch_ranks(n, sys.argv[1:]))
    args.gpus = n
    # a rank that never joins a library collective ends the run in a minute (the library aborts the
    # communicator and raises) instead of the default five
    os.environ.setdefault("SRHIP_COMM_TIMEOUT_S", "60")
    if args.launch_check:
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "world": n,
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
        return
    if args.config == "c4":
        if n > 1:
            raise SystemExit("bench.py: --config c4 is a one-GPU configuration (BASELINE.json C4)")
        return bench_c4(args)
    if args.config in ("c1", "c3"):
        return bench_search(args)
    if args.mode == "rowshard":
        return bench_rowshard(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        # torch first: libsrhip then binds to the already-loaded HIP runtime (same soname)
        import torch
        import torch.distributed as dist

        # (rehearsal on fewer GPUs than ranks: SRHIP_BENCH_BACKEND=gloo, ranks share devices round-robin)
        backend = os.environ.get("SRHIP_BENCH_BACKEND", "nccl")
        if backend != "nccl":
            local_rank %= max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_rank)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    red_dev = f"cuda:{local_rank}" if os.environ.get("SRHIP_BENCH_BACKEND", "nccl") == "nccl" else "cpu"

    import numpy as np

    import srhip

    from srhip import workloads

    opts, X, y, trees, nodes, offs = workloads.c2(rank, args.ntrees, args.rows,
                                                  tuple(o for o in args.binops.split(",") if o),
                                                  tuple(o for o in args.unaops.split(",") if o))
    nfeat, n = X.shape

    ctx = srhip.get_context(local_rank)
    ds = srhip.DeviceDataset(ctx, X, y)
    loss = srhip.L2DistLoss()
    t0 = time.perf_counter()
    prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
    compile_ms = (time.perf_counter() - t0) * 1e3
    st = prog.stats()
    nodes_total, ops_total = st["total_nodes"], st["total_opnodes"]
    work = nodes_total * n                    # tree-node x row evaluations per step
    flops = (ops_total + 3 * args.ntrees) * n  # 1 flop / operator node / row + 3 (fused L2)

    def barrier():
        ctx.synchronize()
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        prog.eval_loss(ds, loss)
    from srhip import parallel

    native = _native_comm(ctx, dist)
    selfcheck = None
    if native is not None:
        # the library's RCCL exchange against torch.distributed's on the same payload, once, before the
        # timed steps: every rank must receive byte-identical migrants from both, else the run uses the
        # torch exchange (and says so in the line)
        l0, _ = prog.eval_loss(ds, loss)

        def _cmp():
            a = native.migrate_topk(nodes, offs, l0, args.migrate_k, 30)
            b = parallel.migrate_topk(nodes, offs, l0, args.migrate_k, 30)
            return parallel.same_migrants(a, b)

        native, selfcheck = _native_selfcheck(native, dist, red_dev, _cmp, "migration payload")

    # islands: every step's evaluation is followed by the migration exchange of its results (the
    # best args.migrate_k trees of every rank reach every rank: one all_gather_into_tensor over
    # RCCL), issued in flight and collected after the next step's evaluation -- the all-gather runs
    # on the collective's stream while the interpreter runs on the library's; the last one is
    # collected inside the timed region
    # The step is one whole population evaluation (probe, persistent launch, precise pass, reduction,
    # losses and did_succeed flags on the host).  Populations are scored back to back the way the
    # search issues them (SingleIteration.jl:112 per population, populations in flight together):
    # step k + 1 is submitted (srhip_eval_loss_submit) before step k's results are waited for, so its
    # launches queue behind step k's while the host takes step k's records and decisions.  Every step
    # is evaluated in full; nothing carries over between them.  --sync times one blocking
    # srhip_eval_loss per step instead; the other figure is reported in extra either way.
    depth = 1 if args.sync else max(2, args.depth)
    barrier()
    parallel.timer.reset()
    t0 = time.perf_counter()
    kms, works = [], []
    pending = None
    inflight = []

    def retire():
        nonlocal pending
        l, ok = inflight.pop(0).wait()
        kms.append(ctx.last_kernel_ms())
        works.append(ctx.last_work())
        if dist is not None:
            if pending is not None:
                pending.wait()
            if native is not None:  # libsrhip's RCCL communicator (srhip_comm_migrate_start)
                pending = native.migrate_start(nodes, offs, l, args.migrate_k, 30)
            else:
                pending = parallel.migrate_topk_async(nodes, offs, l, args.migrate_k, 30)
        return l, ok

    for _ in range(args.steps):
        inflight.append(prog.eval_loss_submit(ds, loss) if depth > 1 else _Done(prog.eval_loss(ds, loss)))
        if len(inflight) >= depth:
            l, ok = retire()
    while inflight:
        l, ok = retire()
    if pending is not None:
        pending.wait()
    barrier()
    dt = time.perf_counter() - t0
    coll_s, coll_calls = parallel.timer.seconds, parallel.timer.calls
    # work COUNTED on the device: the rows each tree was actually evaluated on (a failed tree -- the
    # reference's early return -- stops at its failing tile and is skipped by later row blocks)
    done_node_rows = float(sum(w["node_rows"] for w in works))
    done_flops = float(sum(w["opnode_rows"] + 3 * w["tree_rows"] for w in works)) / args.steps
    if dist is not None:
        import torch

        tt = torch.tensor([dt], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        tw = torch.tensor([done_node_rows], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tw, op=dist.ReduceOp.SUM)
        done_node_rows = float(tw.item())
    ms_per_step = dt * 1e3 / args.steps
    value = done_node_rows / dt               # evaluated node-rows per second, all ranks
    nominal_value = work * world * args.steps / dt
    kern_ms = float(np.mean(kms))
    achieved = done_flops / (kern_ms * 1e-3) / 1e12

    def timed_steps(pr, pipe=1):
        """(seconds for args.steps evaluations after the warmup, max over ranks; mean kernel ms;
        counted flops per launch; counted node-rows per launch).  pipe = 2: each evaluation submitted
        before the previous one is waited for, as the headline loop does."""
        for _ in range(args.warmup):
            pr.eval_loss(ds, loss)
        barrier()
        t0 = time.perf_counter()
        km, wk, q = [], [], []
        for i in range(args.steps + pipe - 1):
            if i < args.steps:
                q.append(pr.eval_loss_submit(ds, loss) if pipe > 1 else _Done(pr.eval_loss(ds, loss)))
            if len(q) >= pipe or i >= args.steps:
                q.pop(0).wait()
                km.append(ctx.last_kernel_ms())
                wk.append(ctx.last_work())
        barrier()
        d = time.perf_counter() - t0
        if dist is not None:
            import torch

            tt = torch.tensor([d], dtype=torch.float64, device=red_dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            d = float(tt.item())
        fl = float(np.mean([w["opnode_rows"] + 3 * w["tree_rows"] for w in wk]))
        nr = float(np.mean([w["node_rows"] for w in wk]))
        return d, float(np.mean(km)), fl, nr

    # the same population with derived columns forced on (the launch picks the plain program for C2:
    # every node of every tree evaluated by its own instruction, over longer row blocks; DESIGN.md
    # §3.1) -- reported beside it
    # the other step form beside the headline's (synchronous calls vs the submit/wait pipeline)
    dt_alt, kern_alt, _, nr_alt = timed_steps(prog, 1 if depth > 1 else 2)
    step_forms = {
        ("pipelined" if depth > 1 else "synchronous"): {"ms_per_step": ms_per_step, "kernel_ms": kern_ms,
                                                        "value": value, "headline": True},
        ("synchronous" if depth > 1 else "pipelined"): {"ms_per_step": dt_alt * 1e3 / args.steps,
                                                        "kernel_ms": kern_alt,
                                                        "value": nr_alt * world * args.steps / dt_alt,
                                                        "headline": False},
        "note": "synchronous: one blocking srhip_eval_loss per step; pipelined: step k + 1 submitted "
                "(srhip_eval_loss_submit) before step k is waited for",
    }
    nan4 = (float("nan"),) * 4
    dt_grid, kern_grid, fl_grid, nr_grid = nan4
    dt_full, kern_full, fl_full, nr_full = nan4
    # the same population through the round-2 grid launch (row blocks x tree groups, no probe)
    if not args.headline_only:
        os.environ["SRHIP_NO_PERSISTENT"] = "1"
        dt_grid, kern_grid, fl_grid, nr_grid = timed_steps(prog)
        del os.environ["SRHIP_NO_PERSISTENT"]
    # ... and without the early exit of failed trees (every row of every tree evaluated)
    if not args.headline_only:
        os.environ["SRHIP_NO_EARLY_EXIT"] = "1"
        dt_full, kern_full, fl_full, nr_full = timed_steps(prog)
        del os.environ["SRHIP_NO_EARLY_EXIT"]

    # trees whose did_succeed needs the precise pass (the bound max|v| x rows reaches half the overflow
    # threshold): srhip_eval_loss runs it for them inside every step
    psums, pchk = prog.eval_loss_partials(ds, loss)
    undecided = int(np.sum(prog.finalize(nfeat, psums, pchk)[2] == 2))

    # end-to-end per population (host compile of 1024 fresh trees + upload + eval)
    t0 = time.perf_counter()
    p2 = srhip.Program(ctx, nodes, offs, opts, np.float32)
    p2.eval_loss(ds, loss)
    e2e_ms = (time.perf_counter() - t0) * 1e3
    p2.close()
    pipeline = None if args.headline_only else population_pipeline(srhip, workloads, ctx, ds, loss, opts, rank, args)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(nodes, offs, opts, X, y, args.cpu_seconds)

    # the kernel variant the library picks for this launch (csrc/srhip_eval.hip pick_rows_per_lane)
    kst = 2 if st["max_stack"] <= 2 else (4 if st["max_stack"] <= 4 else 8)
    rpl = 16 if (kst == 2 and n >= 4096) else 8
    kname = f"srhip::eval_kernel<float, {rpl}, {kst}, 0, true>"
    traffic, valu_issue, traffic_src = pmc_summary(kname)

    if rank == 0:
        out = {
            "metric": "tree-node x row evals/sec (whole node), 1k trees x 1M rows f32; % VALU peak",
            "value": value,
            "unit": "node-row evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (X ~ N(0,1) 5x1M, y = 2cos(x4) + x1^2 - 2 + 0.1 N(0,1); trees from the "
                    "reference's gen_random_tree_fixed_size distribution, sizes U{1..30})",
            "config": {
                "workload": "C2 eval-only: 1024 random trees (size<=30) x 1M rows x 5 features Float32, fused L2 loss",
                "ntrees_per_gpu": args.ntrees, "rows": n, "features": nfeat,
                "nodes_per_step": int(nodes_total), "opnodes_per_step": int(ops_total),
                "parallelism": f"islands{world}" if world > 1 else "single",
                "trees_ok": int(ok.sum()),
            },
            # N > 1: the per-step migration exchange (parallel.migrate_topk), wall time on rank 0
            "collective": None if dist is None else {
                "op": f"all-gather of each rank's {args.migrate_k} best trees (node tables + losses), "
                      f"in flight during the next step's evaluation",
                "native_selfcheck": selfcheck,
                "backend": "rccl (libsrhip srhip_comm_migrate_start/wait)" if native is not None
                           else f"torch.distributed {dist.get_backend()} all_gather_into_tensor",
                "ranks": world, "calls_per_step": coll_calls / args.steps,
                "ms_per_step": coll_s * 1e3 / args.steps},
            "roofline": {
                "bound": "valu",
                "achieved": achieved,
                "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved / PEAK_FP32_TFLOPS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "kernel": kname,
                # HIP events around the step's interpreter launches (probe + persistent main launch)
                "kernel_ms": kern_ms,
                "launches_per_step": 2,
                # counted on the device (srhip_last_work): evaluated operator-node rows + 3 x tree-rows
                "flops_per_launch": int(done_flops),
                "nominal_flops_per_launch": int(flops),
                # SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE x 1024 SIMDs) from the same PMC summary:
                # the issue-slot bound the kernel actually runs against
                "valu_issue_util": valu_issue,
                "op_mix": op_mix(nodes, opts),
            },
            "cpu_baseline": cpu,
            "extra": {
                "compile_ms_1024_trees": compile_ms, "end_to_end_ms_per_population": e2e_ms,
                "population_pipeline": pipeline,
                "step_forms": step_forms,
                "undecided_trees_per_step": undecided,
                # population scoring rate: every live tree's nodes x every row per step / step time (the
                # rows a failed tree skipped counted as if evaluated)
                "nominal_value": nominal_value,
                "evaluated_fraction": done_node_rows / (work * world * args.steps),
                "grid_launch": {"value": nr_grid * world * args.steps / dt_grid, "kernel_ms": kern_grid,
                                "frac": fl_grid / (kern_grid * 1e-3) / 1e12 / PEAK_FP32_TFLOPS,
                                "nominal_value": work * world * args.steps / dt_grid,
                                "note": "SRHIP_NO_PERSISTENT=1: the round-2 launch (row blocks x tree groups)"},
                "no_early_exit": {"value": nr_full * world * args.steps / dt_full, "kernel_ms": kern_full,
                                  "frac": fl_full / (kern_full * 1e-3) / 1e12 / PEAK_FP32_TFLOPS,
                                  "note": "SRHIP_NO_EARLY_EXIT=1: failed trees evaluated on every row"},
            },
        }
        print(json.dumps(out))
    if native is not None:
        native.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def population_pipeline(srhip, workloads, ctx, ds, loss, opts, rank, args, npop=10):
    """Fresh populations through the whole boundary (SURVEY.md section 8 row f1's producer side): host
    compile (no code-cache hits: every population is new trees), upload and fused-loss evaluation of
    `npop` C2-shaped populations, (a) one after another and (b) pipelined -- population i + 1
    compiled on a host thread while population i evaluates (both calls release the interpreter
    lock) -- plus the compile of a population seen before (per-tree code-cache hits)."""
    import concurrent.futures as cf
    import gc

    import numpy as np

    # every population set is generated up front: generating one takes host seconds, and a device left
    # idle that long drops its clocks (the timed sections each start after ~50 ms of evaluations)
    def gen(seed0):
        return [workloads.c2(rank + seed0 + i, args.ntrees, 4096)[4:] for i in range(npop + 1)]

    pops, pops_pipe, pops_two, pops_async = gen(1000), gen(2000), gen(3000), gen(4000)

    def make(i):
        return srhip.Program(ctx, pops[i][0], pops[i][1], opts, np.float32)

    hot = make(npop)  # warm-up (thread pool, allocations) on a population the timed ones do not share
    hot.eval_loss(ds, loss)

    def steady_clocks():
        for _ in range(40):
            hot.eval_loss(ds, loss)

    comp = []
    for i in range(npop // 2):
        t0 = time.perf_counter()
        p = make(i)
        comp.append(time.perf_counter() - t0)
        p.close()
    make(0).close()  # the same trees a second time: the cache makes their entries
    t0 = time.perf_counter()
    p = make(0)  # and a third: code-cache hits
    warm = time.perf_counter() - t0
    p.close()
    # the timed sections run with the interpreter's cyclic garbage collector paused (as timeit does): a
    # full collection over the process's objects is a ~10 ms pause unrelated to the workload
    gc.collect()
    gc.disable()
    steady_clocks()
    seq, seq_k = [], []
    for i in range(npop // 2, npop):
        t0 = time.perf_counter()
        p = make(i)
        p.eval_loss(ds, loss)
        seq.append(time.perf_counter() - t0)
        seq_k.append(ctx.last_kernel_ms())
        p.close()
    # pipelined over fresh populations (new seeds: no cache hits)
    pops[:] = pops_pipe
    steady_clocks()
    with cf.ThreadPoolExecutor(1) as ex:
        # the pipeline's steady state: timed from the moment the first program is ready (its compile is
        # the one-time fill, reported apart) to the last population's results
        tf = time.perf_counter()
        fut = ex.submit(make, 0)
        p = fut.result()
        t0 = time.perf_counter()
        fill = t0 - tf
        ph_eval, ph_wait, pipe_k = [], [], []
        for i in range(npop):
            if i + 1 < npop:
                fut = ex.submit(make, i + 1)
            ta = time.perf_counter()
            p.eval_loss(ds, loss)
            pipe_k.append(ctx.last_kernel_ms())  # this population's own interpreter launches (HIP events)
            p.close()
            tb = time.perf_counter()
            if i + 1 < npop:
                p = fut.result()
            ph_eval.append(tb - ta)
            ph_wait.append(time.perf_counter() - tb)
        pipe_sync = (time.perf_counter() - t0) / npop
    # (b') the same pipeline through srhip_eval_loss_submit / _wait: population i + 1's launches are queued
    # on the stream behind population i's before i's results are waited for, so the device does not idle
    # through i's wait, decisions and teardown or i + 1's launch sequence
    pops[:] = pops_async
    steady_clocks()
    with cf.ThreadPoolExecutor(1) as ex:
        tf = time.perf_counter()
        p = ex.submit(make, 0).result()
        t0 = time.perf_counter()
        fill_async = t0 - tf
        fut = ex.submit(make, 1) if npop > 1 else None
        tk = p.eval_loss_submit(ds, loss)
        async_k, async_it = [], []
        for i in range(npop):
            ta = time.perf_counter()
            nxt = tk_next = None
            if i + 1 < npop:
                nxt = fut.result()
                if i + 2 < npop:
                    fut = ex.submit(make, i + 2)
                tk_next = nxt.eval_loss_submit(ds, loss)
            tk.wait()
            async_k.append(ctx.last_kernel_ms())  # population i's own launches (its result set's events)
            p.close()
            p, tk = nxt, tk_next
            async_it.append(time.perf_counter() - ta)
        pipe = (time.perf_counter() - t0) / npop
    # (c) two evaluation streams: one compile thread builds the populations in order, alternately for
    # two contexts (own stream, slabs and block counter each; programs upload on the context's upload
    # stream; the dataset is shared); one host thread per context evaluates its populations.  A
    # population's launch, wait and decisions overlap the other context's kernels, which queue behind
    # each other on the CUs.
    import queue

    pops[:] = pops_two
    nstream = max(2, int(os.environ.get("SRHIP_BENCH_STREAMS", "2")))
    ctxs = [ctx] + [srhip.Context(ctx.device) for _ in range(nstream - 1)]
    for c in ctxs[1:]:  # each extra context's first launch (allocations) outside the timing
        q = srhip.Program(c, pops[npop][0], pops[npop][1], opts, np.float32)
        q.eval_loss(ds, loss)
        q.close()
    ready = [queue.Queue() for _ in ctxs]

    def produce():
        for i in range(npop):
            ready[i % nstream].put(srhip.Program(ctxs[i % nstream], pops[i][0], pops[i][1], opts, np.float32))
        for r in ready:
            r.put(None)

    def consume(k):
        while True:
            q = ready[k].get()
            if q is None:
                return
            q.eval_loss(ds, loss)
            q.close()

    steady_clocks()
    with cf.ThreadPoolExecutor(1 + nstream) as ex:
        t0 = time.perf_counter()
        futs = [ex.submit(produce)] + [ex.submit(consume, k) for k in range(nstream)]
        for f in futs:
            f.result()
        pipe2 = (time.perf_counter() - t0) / npop
    gc.enable()
    for c in ctxs[1:]:
        c.close()
    hot.close()
    return {"populations": npop, "trees_each": args.ntrees,
            "compile_ms_fresh": 1e3 * float(np.median(comp)), "compile_ms_cached": 1e3 * warm,
            "sequential_ms_per_population": 1e3 * float(np.mean(seq)),
            # pipelined: compile on a host thread + srhip_eval_loss_submit / _wait (the next population's
            # launches queued behind the current one's); pipelined_sync: the same with srhip_eval_loss
            "pipelined_ms_per_population": 1e3 * pipe, "pipeline_fill_ms": 1e3 * fill_async,
            "pipelined_kernel_ms": float(np.mean(async_k)),
            "pipelined_kernel_ms_each": [round(k, 3) for k in async_k],
            "pipelined_over_kernel_ms": 1e3 * pipe - float(np.mean(async_k)),
            "pipelined_iterations_ms": [round(1e3 * a, 3) for a in async_it],
            "pipelined_sync_ms_per_population": 1e3 * pipe_sync, "pipelined_sync_fill_ms": 1e3 * fill,
            # the fresh populations are other random trees than the headline's: their own launches
            # (probe + persistent, HIP events) are the like-for-like kernel time of each section
            "sequential_kernel_ms": float(np.mean(seq_k)), "pipelined_sync_kernel_ms": float(np.mean(pipe_k)),
            "pipelined_sync_over_kernel_ms": 1e3 * pipe_sync - float(np.mean(pipe_k)),
            "pipelined_phases_ms": {"eval_close": 1e3 * float(np.median(ph_eval)),
                                    "wait_next": 1e3 * float(np.median(ph_wait)),
                                    "iterations": [round(1e3 * (a + b), 3) for a, b in zip(ph_eval, ph_wait)],
                                    "eval_close_each": [round(1e3 * a, 3) for a in ph_eval]},
            "two_stream_ms_per_population": 1e3 * pipe2, "streams": nstream,
            "note": "compile + upload + srhip_eval_loss per fresh 1024-tree population (the Python garbage collector paused in the timed sections); pipelined: the next "
                    "population compiled on a host thread during the current evaluation, steady state (the "
                    "first population's compile is the pipeline's fill, timed apart); two_stream: one compile "
                    "thread, populations alternating between two contexts each evaluated by its own host "
                    "thread, wall time of all populations (compile fill included) / npop"}


def _native_comm(ctx, dist):
    """libsrhip's own RCCL communicator for the ranks' exchanges (parallel.NativeComm) when the ranks
    run on distinct GPUs under the nccl backend; None otherwise (single rank, the gloo rehearsals on
    one GPU -- RCCL cannot place two ranks on one device -- or SRHIP_BENCH_COMM=torch), and the
    torch.distributed exchange is used."""
    if dist is None or os.environ.get("SRHIP_BENCH_BACKEND", "nccl") != "nccl":
        return None
    if os.environ.get("SRHIP_BENCH_COMM", "native") != "native":
        return None
    from srhip import parallel

    try:
        return parallel.NativeComm.from_process_group(ctx)
    except Exception as e:  # pragma: no cover - reported, the torch path takes over
        print(f"[bench] native RCCL communicator unavailable ({e}); using torch.distributed", file=sys.stderr)
        return None


def _native_selfcheck(native, dist, red_dev, compare, what):
    """Run compare() -- the native exchange against torch.distributed's on one payload -- on every rank;
    keep the native communicator only if every rank saw identical results.  (native or None, note)."""
    import torch

    try:
        same = bool(compare())
        err = None
    except Exception as e:  # an RCCL error or the library's collective timeout: fall back, reported
        same, err = False, str(e)
    flag = torch.tensor([1 if same else 0], dtype=torch.int32, device=red_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if int(flag.item()) == 1:
        return native, f"native == torch.distributed ({what}, every rank)"
    native.close()
    note = f"native != torch.distributed ({what}{': ' + err if err else ''}); torch.distributed exchange used"
    print(f"[bench] {note}", file=sys.stderr)
    return None, note


def bench_rowshard(args):
    """c2 --mode rowshard: ONE population of 1024 random trees over the C3-shape dataset (10 features
    x 10M rows F32, workloads.c3_shard), its rows sharded over the ranks (SURVEY.md 8(e) "very large
    row counts"): a step = srhip_eval_loss_partials on this rank's rows + the fused all-reduce of the
    per-tree partials (parallel.allreduce_partials: SUM / MAX over RCCL) + the did_succeed decision,
    identical on every rank.  Strong scaling: the total work is fixed."""
    import numpy as np

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    backend = os.environ.get("SRHIP_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local_rank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    import srhip
    from srhip import parallel, workloads

    n = 10_000_000 if args.rows == 1_000_000 else args.rows
    lo, hi = parallel.shard_rows(n, rank, world)
    X, y = workloads.c3_shard(lo, hi)
    opts, trees, nodes, offs = workloads.rowshard_population(args.ntrees)
    ctx = srhip.get_context(local_rank)
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
    loss = srhip.L2DistLoss()
    st = prog.stats()
    nfeat = X.shape[0]

    native = _native_comm(ctx, dist)
    selfcheck = None
    if native is not None:  # the library's sharded evaluation against the torch.distributed path, once
        red_dev = f"cuda:{local_rank}" if backend == "nccl" else "cpu"

        def _cmp():
            a = native.eval_loss_sharded(prog, ds, loss)
            b = parallel.eval_loss_sharded(prog, nfeat, lambda: prog.eval_loss_partials(ds, loss),
                                           precise=lambda tr: prog.eval_precise_partials(ds, tr))
            return (np.asarray(a[0], np.float64).tobytes() == np.asarray(b[0], np.float64).tobytes()
                    and np.array_equal(a[1], b[1]))

        native, selfcheck = _native_selfcheck(native, dist, red_dev, _cmp, "sharded losses and did_succeed")

    def step():
        if native is not None:  # srhip_eval_loss_sharded: partials, RCCL all-reduce, decision in the library
            return native.eval_loss_sharded(prog, ds, loss)
        return parallel.eval_loss_sharded(prog, nfeat, lambda: prog.eval_loss_partials(ds, loss),
                                          precise=lambda tr: prog.eval_precise_partials(ds, tr))

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    dist.barrier()
    parallel.timer.reset()
    n0 = native.stats()[1] if native is not None else 0.0
    t0 = time.perf_counter()
    kms, done = [], 0.0
    for _ in range(args.steps):
        l, ok = step()
        kms.append(ctx.last_kernel_ms())
        done += ctx.last_work()["node_rows"]
    ctx.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    # the exchanges alone: the library's own clock around its RCCL group (issue -> completion seen), or
    # the torch path's timer around its all-reduces
    coll_s = (native.stats()[1] - n0) * 1e-3 if native is not None else parallel.timer.seconds
    red = torch.device("cuda", local_rank) if backend == "nccl" else torch.device("cpu")
    tt = torch.tensor([dt, coll_s, float(np.mean(kms))], dtype=torch.float64, device=red)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    tw = torch.tensor([done], dtype=torch.float64, device=red)
    dist.all_reduce(tw, op=dist.ReduceOp.SUM)
    dt, coll_max, kern_max = (float(v) for v in tt.cpu().numpy())
    if rank == 0:
        print(json.dumps({
            "metric": "tree-node x row evals/sec (whole node), 1k trees x 10M rows f32 row-sharded over the ranks",
            "value": float(tw.item()) / dt, "unit": "node-row evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (X ~ N(0,1) 10 x 10M in seeded 2^20-row chunks, C3's formula for y)",
            "config": {"workload": f"rowshard: {args.ntrees} random trees (size<=30) x {n} rows x 10 features F32, "
                                   f"rows split over {world} rank(s), fused L2",
                       "rows_per_rank": hi - lo, "nodes": int(st["total_nodes"]), "parallelism": f"rowshard{world}",
                       "trees_ok": int(ok.sum())},
            "nominal_value": st["total_nodes"] * n * args.steps / dt,
            "kernel_ms_max_over_ranks": kern_max,
            "collective": {"op": "all_reduce SUM (per-tree loss sums, feature stats) + all_reduce MAX (check "
                                 "statistics) on one buffer",
                           "backend": "rccl (libsrhip srhip_eval_loss_sharded)" if native is not None
                                      else f"torch.distributed {dist.get_backend()}", "ranks": world,
                           "native_selfcheck": selfcheck,
                           "ms_per_step_max_over_ranks": coll_max * 1e3 / args.steps},
        }))
    if native is not None:
        native.close()
    dist.barrier()
    dist.destroy_process_group()


def pmc_summary(kname, pattern="*pmc_c2*.json"):
    """The committed rocprofv3 --pmc summary of this same command for the kernel `kname`
    (scripts/pmc.sh / pmc_grad.sh + scripts/pmc_summary.py --json; separate counter passes,
    FETCH_SIZE doubled per MI355X_MICROARCH.md): (HBM bytes per launch, VALU issue utilisation,
    source file).  Nones if no summary for this kernel variant is committed."""
    import glob

    # the newest round's final summary when committed (file names sort by build, not by date), else
    # the last by name
    finals = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern.replace("*", "r[0-9][0-9]_", 1)
                                           .replace("*", "_final"))))
    files = finals[-1:] if finals else sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)))
    if not files:
        return None, None, None
    try:
        summ = json.load(open(files[-1]))
    except (OSError, ValueError):
        return None, None, None
    want = kname.replace("srhip::", "").replace(" ", "")
    for k, d in summ.items():
        if want in k.replace(" ", "") and "hbm_bytes" in d:
            return d["hbm_bytes"], d.get("valu_issue_util"), os.path.relpath(files[-1], ROOT)
    return None, None, None


def op_mix(nodes, opts):
    """Operator-node counts of the population by operator name (report the op mix
    beside the flop fraction — a transcendental is one algorithmic flop but ~20 VALU issues)."""
    import collections

    c = collections.Counter()
    for nd in nodes:
        if nd["degree"] == 1:
            c[opts.unary_operators[nd["op"] - 1]] += 1
        elif nd["degree"] == 2:
            c[opts.binary_operators[nd["op"] - 1]] += 1
    return dict(c)


def cpu_baseline(nodes, offs, opts, X, y, target_s):
    """The oracle (C restatement of the reference's array-at-a-time evaluator, OpenMP across
    trees like the reference's per-population tasks) on a bounded row sample of the same
    population, scaled to ~target_s seconds."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    threads = min(threads, os.cpu_count() or 1)
    nodes_total = int(offs[-1])
    m = 4096
    t0 = time.perf_counter()
    oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X[:, :m].copy(), y[:m].copy(),
                           nthreads=threads)
    t1 = time.perf_counter() - t0
    m2 = int(min(X.shape[1], max(m, m * target_s / max(t1, 1e-6))))
    Xs, ys = X[:, :m2].copy(), y[:m2].copy()
    t0 = time.perf_counter()
    _, _, _, used = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, Xs, ys, nthreads=threads)
    dt = time.perf_counter() - t0
    # the work definition of `value`: node-rows actually evaluated -- the oracle stops a failed tree at
    # its first failed check (DynamicExpressions' early return) as the device stops it at its failing tile
    done = oracle.eval_loss_batch.last_node_rows
    return {
        "value": done / dt,
        "unit": "node-row evals/s",
        "cores": int(used),
        "kind": "port",
        "nominal_value": nodes_total * m2 / dt,
        "evaluated_fraction": done / (nodes_total * m2),
        "sample": f"all {len(offs) - 1} trees x first {m2} of the 1M rows ({dt:.1f} s), oracle/sr_oracle.c "
                  f"array-at-a-time restatement, OpenMP over trees on {int(used)} threads (the job's core "
                  f"allotment); value counts the node-rows evaluated before each failed tree's early return",
    }


def bench_c4(args):
    """C4: optimize_constants (BFGS(8 iterations) + 2 restarts, src/ConstantOptimization.jl) on 512
    fixed-size-20 trees with >= 2 constants over 5 x 100k Float64 rows, one MI355X.  A step = one
    batched srhip_optimize_constants from the same initial constants.  Also reports the
    dual-number gradient launch alone (node-row evals/s of the loss + gradient)."""
    import numpy as np

    import srhip

    from srhip import workloads

    rows = 100_000 if args.rows == 1_000_000 else args.rows
    ntrees = 512 if args.ntrees == 1024 else args.ntrees
    opts, X, y, trees, nodes, offs = workloads.c4(ntrees, rows)
    ctx = srhip.get_context(0)
    ds = srhip.DeviceDataset(ctx, X, y)
    prog = srhip.Program(ctx, nodes, offs, opts, np.float64)
    x0 = np.concatenate(prog.get_constants())
    loss = srhip.L2DistLoss()
    base, ok = prog.eval_loss(ds, loss)

    def step():
        prog.set_constants(x0)
        return prog.optimize_constants(ds, loss, iterations=8, nrestarts=2, seed=7)

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, improved, fcalls = step()
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    # gradient launch alone (all 512 trees' loss + d loss / d c), HIP events around the dual-number
    # kernel on the library's stream
    st = prog.stats()
    for _ in range(3):
        prog.eval_loss_grad(ds, loss)
    ctx.synchronize()
    t0 = time.perf_counter()
    gkms = []
    for _ in range(10):
        prog.eval_loss_grad(ds, loss)
        gkms.append(ctx.last_kernel_ms())
    gdt = (time.perf_counter() - t0) / 10
    gk_ms = float(np.mean(gkms))
    # algorithmic flops of one gradient launch: per row, every operator node costs its
    # value plus one chain-rule product per constant of the tree; the fused loss 3 + 2 per constant
    nconst = prog.num_constants().astype(np.int64)
    opn = np.array([int(np.sum(nodes[offs[t]:offs[t + 1]]["degree"] > 0)) for t in range(len(offs) - 1)])
    gflops = float(rows * np.sum(opn * (1 + nconst) + 3 + 2 * nconst))
    cpu = None if args.no_cpu else cpu_c4_baseline(nodes, offs, opts, X, y, args.cpu_seconds)
    fin = np.isfinite(base)
    # HBM bytes of the profiled gradient variant (scripts/pmc_grad.sh over scripts/grad_bench.py: the
    # same 512 x 100k population, one full loss + gradient launch)
    gname = "srhip::grad_kernel<double, 4, 2, 0, true, 2>"
    gtraffic, gvalu, gsrc = pmc_summary(gname, "*pmc_grad_c4*.json")
    print(json.dumps({
        "metric": "C4 batched constant optimisation: wall time per optimize_constants over the population",
        "value": dt * 1e3, "unit": "ms", "higher_is_better": False, "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt * 1e3, "dtype": "f64", "data": "synthetic (X ~ N(0,1) 5x100k; fixed-size-20 trees, >= 2 consts)",
        "config": {"workload": f"C4: {ntrees} trees x {rows} rows Float64, BFGS(8) + 2 restarts",
                   "ntrees": ntrees, "rows": rows, "nodes": int(st["total_nodes"])},
        "objective_evals_per_s": float(np.sum(fcalls)) / dt,
        "improved_trees": int(improved.sum()),
        "mean_loss_before": float(np.mean(base[fin])), "mean_loss_after": float(np.mean(out[fin])),
        # the mean is dominated by a few overflow-scale losses; the median shows the typical tree
        "median_loss_before": float(np.median(base[fin])), "median_loss_after": float(np.median(out[fin])),
        # a tree whose loss stays at ~1e250 fixes the arithmetic mean: the log-mean shows the whole population
        "mean_log10_loss_before": float(np.mean(np.log10(np.maximum(base[fin], 1e-300)))),
        "mean_log10_loss_after": float(np.mean(np.log10(np.maximum(out[fin], 1e-300)))),
        "grad_launch_ms": gdt * 1e3,
        "grad_node_row_evals_per_s": st["total_nodes"] * rows / gdt,
        "roofline": {"bound": "valu", "kernel": "srhip::grad_kernel<double, KT, K, 0>", "kernel_ms": gk_ms,
                     "flops_per_launch": gflops, "achieved": gflops / (gk_ms * 1e-3) / 1e12,
                     "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                     "frac": gflops / (gk_ms * 1e-3) / 1e12 / PEAK_FP64_TFLOPS, "traffic": gtraffic,
                     "traffic_kernel": gname if gtraffic is not None else None, "traffic_source": gsrc,
                     "valu_issue_util": gvalu},
        "cpu_baseline": cpu,
    }))


def _c4_cpu_worker(job):
    """cpu_c4_baseline's pool task: optimise trees one after another until the deadline."""
    nodes, offs, trees, binops, unaops, X, y, deadline = job
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import optim

    done = 0
    for t in trees:
        if time.time() > deadline:
            break
        tn = nodes[offs[t]:offs[t + 1]].copy()
        optim.optimize_constants(tn, binops, unaops, X, y, iterations=8, nrestarts=2,
                                 rng=np.random.default_rng(int(t)))
        done += 1
    return done


def cpu_c4_baseline(nodes, offs, opts, X, y, target_s):
    """The reference procedure (oracle/optim.py: finite-difference BFGS / Newton + BackTracking,
    iterations 8, 2 restarts) over the population's trees on ALL the host cores this job may use
    (a process pool over trees, as the reference's :multithreading spreads populations over
    threads), for about target_s seconds; ms per optimize_constants of the whole population,
    extrapolated from the trees finished."""
    import multiprocessing as mp

    import numpy as np

    cores = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1), os.cpu_count() or 1)
    order = np.random.default_rng(3).permutation(len(offs) - 1)
    chunks = [order[i::cores] for i in range(cores)]
    t0 = time.perf_counter()
    deadline = time.time() + target_s
    # spawned workers (the parent may already hold the GPU: no fork of its state)
    with mp.get_context("spawn").Pool(cores) as pool:
        done = sum(pool.map(_c4_cpu_worker, [(nodes, offs, c, opts.binop_codes, opts.unaop_codes, X, y, deadline)
                                             for c in chunks]))
    dt = time.perf_counter() - t0
    return {"value": dt / max(done, 1) * (len(offs) - 1) * 1e3 * 1.0, "unit": "ms", "cores": cores, "kind": "port",
            "sample": f"{done} of the {len(offs) - 1} trees in {dt:.1f} s on {cores} worker processes (one tree per "
                      f"process at a time), oracle/optim.py finite-difference BFGS/Newton(8) + 2 restarts over the C "
                      f"oracle's eval_loss; whole-population time extrapolated from the trees finished"}


def bench_search(args):
    """C1 / C3: the full search (srhip.search.equation_search: regularized-evolution islands,
    every score through the device coalescer, constants optimised on the device).
      c1: README example, X = randn(2, 100) Float64, y = 2cos(x2) + x1^2 - 2, + * / - cos exp,
          populations = 20 (the config's niterations = 40; default here a bounded 2).
      c3: 10 x 10M Float32, populations = 15 per GPU, islands sharded over the ranks with the
          per-iteration all-gather migration (RCCL under torch.distributed.run).
    value = tree-node x row evaluations scored per second (all ranks), the search's wall time
    bracketed by barriers, max over ranks.  cpu_baseline (rank 0, N = 1): the same search with
    the oracle as scorer (c1), or the oracle's population-eval rate on a row sample (c3)."""
    import numpy as np

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    import srhip
    from srhip import search as S

    c1 = args.config == "c1"
    ops = dict(binary_operators=("+", "*", "/", "-"), unary_operators=("cos", "exp"))
    if c1:
        rng = np.random.default_rng(0)
        X = rng.standard_normal((2, 100))
        y = 2 * np.cos(X[1]) + X[0] ** 2 - 2
        npops, iters = 20, args.iterations or 2
    else:
        from srhip import workloads

        n = 10_000_000 if args.rows == 1_000_000 else args.rows
        X, y = workloads.c3_data(n)  # same dataset on every rank (replicas)
        npops, iters = 15 * world, args.iterations or 1
    kw = dict(populations=npops, deterministic=True, seed=1, device=local_rank, **ops)
    if args.ncycles:
        kw["ncycles_per_iteration"] = args.ncycles
    opts = srhip.Options(**kw)
    d = srhip.Dataset(X, y)
    if dist is not None:
        dist.barrier()
    mp = args.parallelism == "multiprocessing"
    procs = args.procs or min(npops // world, 16)
    skw = dict(parallelism=args.parallelism, procs=procs, devices=[local_rank]) if mp else {}
    t0 = time.perf_counter()
    res = S.equation_search(d, None, opts, niterations=iters, **skw)
    dt = time.perf_counter() - t0
    if dist is not None:
        import torch

        tt = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    front = res.pareto_frontier()
    best = float(min(m.loss for m in front))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_search_baseline(args, c1, X, y, opts, iters, dt, skw)
    if rank == 0:
        print(json.dumps({
            "metric": ("C1 equation_search (README example)" if c1 else "C3 equation_search 10M x 10 F32 islands")
                      + ": tree-node x row evals/s",
            "value": res.node_rows / dt, "unit": "node-row evals/s", "higher_is_better": True,
            "n_gpus": world, "steps": iters, "warmup": 0, "ms_per_step": dt * 1e3 / iters,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64" if c1 else "f32",
            "data": "synthetic (README formula)" if c1 else "synthetic (X ~ N(0,1) 10x10M, fixed 10-feature formula)",
            "config": {"workload": ("C1: X=randn(2,100) F64, + * / - cos exp, populations=20" if c1 else
                                    f"C3: 10M rows x 10 features F32, {npops} populations ({npops // world} per GPU)"),
                       "iterations": iters, "populations": npops, "ncycles_per_iteration": S.search_option(opts, "ncycles_per_iteration"),
                       "parallelism": (f"islands{world}" if world > 1 else "single")
                                      + (f", {procs} worker processes per GPU" if mp else ", island threads")},
            "search": {"wall_s": dt, "num_evals": res.num_evals, "evals_per_s": res.num_evals / dt,
                       "node_rows": res.node_rows, "best_loss": best,
                       "baseline_loss": float(np.mean((y.astype(np.float64) - y.mean()) ** 2)),
                       "coalescer": res.coalescer_stats,
                       # interpreter time (HIP events) / wall time: how busy the search keeps the GPU;
                       # worker time (compile + upload + launch + wait) / wall time
                       "device_busy_frac": res.coalescer_stats.get("kernel_ms", 0.0) / (dt * 1e3),
                       "coalescer_busy_frac": res.coalescer_stats.get("busy_ms", 0.0) / (dt * 1e3),
                       "coalesce_wait_us": int(os.environ.get("SRHIP_COALESCE_WAIT_US", "0"))},
            "cpu_baseline": cpu,
        }))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _oracle_scorer_factory(worker, dataset, options):
    """cpu_baseline legs of c1 / c3: each worker process scores with the oracle (bench only)."""
    return _OracleScorer(dataset, options)


class _OracleScorer:
    """score_func through the oracle, and optimize_constants through oracle/optim.py's reference
    procedure (finite-difference BFGS / Newton + BackTracking) -- the search's whole host-side
    workload on the CPU (bench cpu_baseline only)."""

    def __init__(self, d, o):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle

        self.d, self.o, self.node_rows, self.orc = d, o, 0, oracle

    def score(self, tree, complexity=None, idx=None):
        import srhip

        nodes, offs = srhip.flatten([tree], self.o, self.d.X.dtype)
        le, _, ok, _ = self.orc.eval_loss_batch(nodes, offs, self.o.binop_codes, self.o.unaop_codes,
                                                self.d.X, self.d.y, nthreads=1)
        self.node_rows += len(nodes) * self.d.n
        loss = float(le[0]) if ok[0] else float("inf")
        return srhip.loss_to_score(loss, self.d.use_baseline, self.d.baseline_loss, tree, self.o,
                                   complexity), loss

    def optimize_constants(self, dataset, members, options, rng=None):
        """api.optimize_constants' contract (src/ConstantOptimization.jl:11-81) with the oracle's
        finite-difference optimiser: improved members get the new constants, loss, score, birth."""
        import numpy as np

        import optim
        import srhip
        from srhip.node import set_constants
        from srhip.utils import get_birth_order

        single = not isinstance(members, (list, tuple))
        ml = [members] if single else list(members)
        rng = np.random.default_rng() if rng is None else rng
        ne = 0.0
        L = dataset.loss_type.type
        for m in ml:
            tree = m.tree if hasattr(m, "tree") else m
            nodes, _ = srhip.flatten([tree], options, dataset.X.dtype)
            x, f, improved = optim.optimize_constants(nodes, options.binop_codes, options.unaop_codes, dataset.X,
                                                      dataset.y, iterations=options.optimizer_iterations,
                                                      nrestarts=options.optimizer_nrestarts, rng=rng)
            ne += 1.0
            if not improved:
                continue
            set_constants(tree, x)
            if hasattr(m, "tree"):
                m.loss = L(f)
                m.score = srhip.loss_to_score(m.loss, dataset.use_baseline, dataset.baseline_loss, m, options)
                if hasattr(m, "birth"):
                    m.birth = get_birth_order()
        return (ml[0] if single else ml), ne


def cpu_search_baseline(args, c1, X, y, opts, iters, gpu_dt, skw=None):
    """The same search (options, seed, populations, iterations) with the whole host workload on the
    CPU: every island's iteration in a worker process (the reference's :multiprocessing, over all
    the cores this job may use), scoring with the oracle (oracle/sr_oracle.c) and optimising
    constants with oracle/optim.py's finite-difference reference procedure.  c1 on its 100 rows;
    c3 on the first 100k of the 10M rows (a bounded sample: the oracle's array-at-a-time cost per
    node-row does not depend on the row count).  value = node-rows scored per second (the same
    definition as the device line's)."""
    import numpy as np

    import srhip
    from srhip import search as S

    cores = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1), os.cpu_count() or 1)
    m = X.shape[1] if c1 else min(X.shape[1], 100_000)
    Xs, ys = (X, y) if c1 else (X[:, :m].copy(), y[:m].copy())
    d = srhip.Dataset(Xs, ys)
    npops = S.search_option(opts, "populations")
    procs = max(1, min(npops, cores))
    t0 = time.perf_counter()
    res = S.equation_search(d, None, opts, niterations=iters, parallelism="multiprocessing", procs=procs,
                            worker_backend="host", scorer_factory=_oracle_scorer_factory)
    dt = time.perf_counter() - t0
    return {"value": res.node_rows / dt, "unit": "node-row evals/s", "cores": procs, "kind": "port",
            "sample": f"the same search ({npops} populations, {iters} iteration(s), seed) over "
                      f"{'all 100' if c1 else f'the first {m} of the {X.shape[1]}'} rows in {procs} worker "
                      f"processes: oracle/sr_oracle.c scores, oracle/optim.py finite-difference constant "
                      f"optimisation, {dt:.1f} s wall"}


if __name__ == "__main__":
    main()
