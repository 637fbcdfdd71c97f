"""Multi-GPU layer: one process per GPU over torch.distributed (backend "nccl" = RCCL over xGMI
on MI355X; "gloo" for the CPU tests).  SURVEY.md 8(e) names two partitions, both here:

* islands (the default, as the reference partitions its populations over workers:
  src/SymbolicRegression.jl:746-793, src/SearchUtils.jl:108-127): every rank holds a full
  dataset replica and its own populations, so evaluation needs no collective at all.  The one
  exchange is migration (src/Migration.jl:16-38 applied on the head node at
  src/SymbolicRegression.jl:933-943): each rank's best members travel as node tables through
  :func:`allgather_trees` (all-gather of a few KB; latency-bound on xGMI).
* row shards (datasets too tall for one device): every rank evaluates every tree on its block
  of rows; :func:`eval_loss_sharded` all-reduces the per-tree partials (sums by SUM, the check
  statistic by MAX for Float32) and every rank takes the did_succeed decision identically
  (include/srhip.h "row-sharded evaluation").  One fused all-reduce per population, plus one
  more only when a tree's overflow check is undecided.

Both exchanges exist twice: natively in libsrhip on RCCL (:class:`NativeComm`, the C ABI's
srhip_comm_* -- what a Julia caller binds), used whenever the ranks run on
distinct GPUs under the nccl backend; and as torch.distributed calls below (the gloo CPU tests and
the one-GPU multi-rank rehearsals, where RCCL cannot place two ranks on one device).
"""
from __future__ import annotations

import numpy as np

from ._lib import NODE_DTYPE


def _dist():
    import torch.distributed as dist

    return dist


def world():
    """(rank, world_size) of the default process group, (0, 1) when not initialised."""
    import sys

    if "torch" not in sys.modules:  # no process group can exist without torch loaded
        return 0, 1
    try:
        dist = _dist()
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank(), dist.get_world_size()
    except ImportError:
        pass
    return 0, 1


def shard_rows(n: int, rank: int, world_size: int):
    """[lo, hi) of rank's contiguous block of n rows (sizes differ by at most one)."""
    base, extra = divmod(n, world_size)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def _device(group=None):
    import torch

    dist = _dist()
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def allreduce_np(a: np.ndarray, op: str = "sum", group=None) -> np.ndarray:
    """All-reduce of a float64 array in place semantics (returns the reduced copy)."""
    import torch

    dist = _dist()
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64).copy()).to(_device(group))
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM, group=group)
    return t.cpu().numpy()


class CollectiveTimer:
    """Wall time spent in this module's collectives (host copies included), for the bench."""

    def __init__(self):
        self.seconds = 0.0
        self.calls = 0

    def reset(self):
        self.seconds, self.calls = 0.0, 0


timer = CollectiveTimer()


_bufs = {}


def _staging(n: int, dtype, dev, role: str):
    """Reused (pinned host, device) buffer pair of n elements for a collective's copies: no allocation
    and no pageable-memory copy per call.  Keyed by role ("partials", "migrate_in", "migrate_out"), so
    a collective's input and output never share a buffer (at world size 1 they have the same size).
    One exchange per role in flight at a time (an async migration is collected before the next is
    issued)."""
    import torch

    key = (role, n, dtype, str(dev))
    if key not in _bufs:
        host = torch.empty(n, dtype=dtype, pin_memory=dev.type == "cuda")
        _bufs[key] = (host, host if dev.type != "cuda" else torch.empty(n, dtype=dtype, device=dev))
    return _bufs[key]


def allreduce_partials(sums: np.ndarray, chk: np.ndarray, chk_op: str, group=None):
    """The row-shard exchange of eval_loss_partials in ONE device buffer [sums | chk] (one host->device
    copy from a reused pinned buffer, the two all-reduces issued back to back on it -- SUM over the
    sums, MAX (Float32) or SUM over the check statistics -- and one copy back).  A non-finite check
    statistic is sent as +Inf, which every backend's MAX keeps (an fmax-style reduction may drop a
    NaN)."""
    import time

    import torch

    dist = _dist()
    t0 = time.perf_counter()
    ns, nc = len(sums), len(chk)
    dev = _device(group)
    host, buf = _staging(ns + nc, torch.float64, dev, "partials")
    hv = host.numpy()
    hv[:ns] = sums
    hv[ns:] = np.where(np.isfinite(chk), chk, np.inf)
    if buf is not host:
        buf.copy_(host, non_blocking=True)
    w1 = dist.all_reduce(buf[:ns], op=dist.ReduceOp.SUM, group=group, async_op=True)
    w2 = dist.all_reduce(buf[ns:], op=dist.ReduceOp.MAX if chk_op == "max" else dist.ReduceOp.SUM, group=group,
                         async_op=True)
    w1.wait()
    w2.wait()
    if buf is not host:
        host.copy_(buf, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
    out = hv.copy()
    timer.seconds += time.perf_counter() - t0
    timer.calls += 1
    return out[:ns], out[ns:]


def eval_loss_sharded(prog, nfeatures: int, partials, precise=None, group=None):
    """Row-sharded eval_loss for every tree of ``prog``.

    partials(): this rank's (sums, chk) — ``prog.eval_loss_partials(shard, loss)`` on a GPU;
    precise(trees): this rank's per-operator sums for undecided trees —
    ``prog.eval_precise_partials(shard, trees)``.  Returns (loss[T], ok[T]) identical on all ranks.
    """
    sums, chk = partials()
    sums, chk = allreduce_partials(sums, chk, "max" if prog.chk_reduce_op() == "max" else "sum", group)
    loss, ok, status = prog.finalize(nfeatures, sums, chk)
    undecided = np.nonzero(status == 2)[0].astype(np.int32)
    if len(undecided):
        if precise is None:
            raise RuntimeError("undecided overflow checks need the precise pass (pass precise=...)")
        opsums = allreduce_np(precise(undecided), "sum", group)
        uok = prog.precise_finalize(undecided, opsums)
        ok[undecided] = uok
        s, wsum = sums[2 * undecided], sums[2 * undecided + 1]
        loss[undecided] = np.where(uok, s / wsum, np.inf)
    return loss, ok


def allgather_trees(nodes: np.ndarray, offsets: np.ndarray, group=None):
    """Migration exchange: every rank's trees (srhip_node tables) -> list of (nodes, offsets) by rank."""
    import torch

    dist = _dist()
    dev = _device(group)
    ws = dist.get_world_size(group)
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    meta = torch.tensor([len(nodes), len(offsets)], dtype=torch.int64, device=dev)
    metas = [torch.zeros_like(meta) for _ in range(ws)]
    dist.all_gather(metas, meta, group=group)
    metas = [m.cpu().numpy() for m in metas]
    maxb = max(int(m[0]) for m in metas) * NODE_DTYPE.itemsize
    maxo = max(int(m[1]) for m in metas)
    buf = np.zeros(maxb + 8 * maxo, dtype=np.uint8)
    raw = nodes.view(np.uint8)
    buf[: len(raw)] = raw
    buf[maxb: maxb + 8 * len(offsets)] = offsets.view(np.uint8)
    t = torch.from_numpy(buf).to(dev)
    outs = [torch.zeros_like(t) for _ in range(ws)]
    dist.all_gather(outs, t, group=group)
    result = []
    for m, o in zip(metas, outs):
        b = o.cpu().numpy()
        nn, no = int(m[0]), int(m[1])
        nd = b[: nn * NODE_DTYPE.itemsize].copy().view(NODE_DTYPE)
        of = b[maxb: maxb + 8 * no].copy().view(np.int64)
        result.append((nd, of))
    return result


def allgather_f64(a: np.ndarray, group=None):
    """Variable-length all-gather of a float64 vector -> list of arrays by rank."""
    import torch

    dist = _dist()
    dev = _device(group)
    ws = dist.get_world_size(group)
    a = np.ascontiguousarray(a, dtype=np.float64).ravel()
    meta = torch.tensor([len(a)], dtype=torch.int64, device=dev)
    metas = [torch.zeros_like(meta) for _ in range(ws)]
    dist.all_gather(metas, meta, group=group)
    lens = [int(m.cpu().numpy()[0]) for m in metas]
    buf = np.zeros(max(1, max(lens)), dtype=np.float64)
    buf[: len(a)] = a
    t = torch.from_numpy(buf).to(dev)
    outs = [torch.zeros_like(t) for _ in range(ws)]
    dist.all_gather(outs, t, group=group)
    return [o.cpu().numpy()[:n].copy() for o, n in zip(outs, lens)]


def exchange_members(trees, scores, losses, options, dtype, group=None):
    """Migration exchange of the island search (src/Migration.jl:16-38 fed from every rank, as the
    reference's head node sees every population's best_sub_pop and the hall of fame,
    src/SymbolicRegression.jl:910-943): this rank's member trees travel as node tables plus
    their (score, loss); returns [(tree, score, loss)] of all ranks in rank order."""
    from .node import flatten, unflatten

    if trees:
        nodes, offs = flatten(trees, options, dtype)
    else:
        nodes, offs = np.zeros(0, dtype=NODE_DTYPE), np.zeros(1, dtype=np.int64)
    sl = np.stack([np.asarray(scores, dtype=np.float64), np.asarray(losses, dtype=np.float64)], 1).ravel()
    got = allgather_trees(nodes, offs, group)
    vals = allgather_f64(sl, group)
    out = []
    for (nd, of), v in zip(got, vals):
        ts = unflatten(nd, of, options) if len(of) > 1 else []
        v = v.reshape(-1, 2)
        out.extend((t, float(v[i, 0]), float(v[i, 1])) for i, t in enumerate(ts))
    return out


def _distinct_devices(ctx, group=None) -> bool:
    """True when every rank of the group runs on a GPU of its own ((host, device) pairs all-gathered, so
    every rank returns the same answer)."""
    import socket

    dist = _dist()
    dev = getattr(ctx, "device", None)
    mine = (socket.gethostname(), int(dev) if dev is not None else -1)
    got = [None] * dist.get_world_size(group)
    dist.all_gather_object(got, mine, group=group)
    return len(set(got)) == len(got)


class IterationExchange:
    """The island search's whole per-iteration exchange as ONE fixed-size all-gather (src/Migration.jl:16-38
    fed from every rank as the reference's head node sees every population's best_sub_pop and the hall of
    fame, src/SymbolicRegression.jl:910-943; the adaptive-parsimony size counts of
    src/SearchUtils.jl RunningSearchStatistics ride along).  Each rank sends one payload

        [nsub, nmembers | offsets (cap + 1) | scores (cap) | losses (cap) | counts (nbin) | node pool]

    of a size every rank computes from the options alone (cap = the most best_sub_pops members a rank
    can hold + one frontier member per complexity; the node pool cap x (maxsize + 1) records), so no
    size round precedes it.  On the nccl backend with ranks on distinct GPUs it travels through
    libsrhip's RCCL communicator (NativeComm.allgather: device buffers, no torch tensors); otherwise
    through one torch.distributed all_gather_into_tensor (gloo CPU tests, one-GPU rehearsals); with
    neither (world size 1, no process group) it is the identity."""

    def __init__(self, cap: int, pool_nodes: int, nbin: int, comm=None, group=None, world: int = 1):
        self.cap, self.pool, self.nbin = int(cap), int(pool_nodes), int(nbin)
        self.comm, self.group, self.world = comm, group, int(world)
        self.head = 8 * (2 + (self.cap + 1) + 2 * self.cap + self.nbin)
        self.last_overflow = None  # (cap, pool) of the last exchange's second round, if it needed one
        self.size = self.head + self.pool * NODE_DTYPE.itemsize

    @classmethod
    def for_search(cls, options, npops: int, world: int, topn: int, nbin: int, make_ctx=None, group=None,
                   native: bool = True):
        """The search's exchange: its capacity from the options; NativeComm (on make_ctx()'s device) when
        native and the process group is nccl -- or no process group exists: world 1 through the library
        -- torch otherwise (SRHIP_SEARCH_COMM=torch forces it)."""
        import os
        import sys

        per_rank = -(-int(npops) // max(1, int(world)))
        maxsize = int(options.maxsize)
        cap = per_rank * int(topn) + maxsize
        comm = None
        use_native = native and make_ctx is not None and os.environ.get("SRHIP_SEARCH_COMM", "native") == "native"
        initialised = "torch" in sys.modules and _dist().is_available() and _dist().is_initialized()
        if use_native and (not initialised or _dist().get_backend(group) == "nccl"):
            ctx = make_ctx()
            if not initialised:
                comm = NativeComm(ctx, 1, 0, NativeComm.unique_id())
            elif _distinct_devices(ctx, group):
                comm = NativeComm.from_process_group(ctx, group)
            # else: ranks share a GPU (a one-GPU nccl rehearsal): RCCL cannot place two ranks on one
            # device, so every rank takes the torch path (the check is collective: all ranks agree)
        return cls(cap, cap * (maxsize + 1), nbin, comm, group, world)

    def needs(self, trees, options, dtype):
        """(members, node records) this rank's payload holds."""
        from .node import flatten

        if not trees:
            return 0, 0
        nodes, _ = flatten(trees, options, dtype)
        return len(trees), len(nodes)

    def pack(self, trees, scores, losses, nsub: int, counts, options, dtype) -> np.ndarray:
        """This rank's payload.  Members or node records past the capacity do not raise here (the other
        ranks are already waiting in the all-gather): the header's member count is written as -1 - n
        with the node count beside it, and exchange() runs a second, larger round on every rank."""
        from .node import flatten

        n = len(trees)
        nodes, offs = flatten(trees, options, dtype) if n else (np.zeros(0, NODE_DTYPE), np.zeros(1, np.int64))
        buf = np.zeros(self.size, dtype=np.uint8)
        h = buf[:self.head].view(np.float64)
        hi = buf[:self.head].view(np.int64)
        c = self.cap
        if n > c or len(nodes) > self.pool:
            hi[0], hi[1], hi[2] = int(nsub), -1 - n, len(nodes)
            return buf
        hi[0], hi[1] = int(nsub), n
        hi[2:2 + n + 1] = offs
        h[3 + c:3 + c + n] = np.asarray(scores, dtype=np.float64)
        h[3 + 2 * c:3 + 2 * c + n] = np.asarray(losses, dtype=np.float64)
        h[3 + 3 * c:3 + 3 * c + self.nbin] = np.asarray(counts, dtype=np.float64)
        buf[self.head:self.head + len(nodes) * NODE_DTYPE.itemsize] = np.ascontiguousarray(nodes).view(np.uint8)
        return buf

    def overflow(self, buf):
        """None, or the (members, node records) an overflowing payload needs."""
        hi = np.asarray(buf, dtype=np.uint8)[:24].view(np.int64)
        return None if hi[1] >= 0 else (int(-1 - hi[1]), int(hi[2]))

    def unpack(self, buf, options):
        """-> (nsub, [(tree, score, loss)], counts)"""
        from .node import unflatten

        buf = np.asarray(buf, dtype=np.uint8)
        h = buf[:self.head].view(np.float64)
        hi = buf[:self.head].view(np.int64)
        c = self.cap
        nsub, n = int(hi[0]), int(hi[1])
        offs = hi[2:2 + n + 1].copy()
        scores, losses = h[3 + c:3 + c + n], h[3 + 2 * c:3 + 2 * c + n]
        counts = h[3 + 3 * c:3 + 3 * c + self.nbin].copy()
        nodes = buf[self.head:self.head + int(offs[-1]) * NODE_DTYPE.itemsize].copy().view(NODE_DTYPE)
        trees = unflatten(nodes, offs, options) if n else []
        return nsub, [(t, float(scores[i]), float(losses[i])) for i, t in enumerate(trees)], counts

    def _gather(self, payload: np.ndarray) -> list:
        """One fixed-size all-gather of payload (the same length on every rank) -> parts by rank."""
        if self.comm is not None:
            return [np.frombuffer(p, dtype=np.uint8) for p in self.comm.allgather(payload.tobytes())]
        if self.world > 1:
            import torch

            dist = _dist()
            dev = _device(self.group)
            size = len(payload)
            host_in, src = _staging(size, torch.uint8, dev, "iter_in")
            host_in.numpy()[:] = payload
            if src is not host_in:
                src.copy_(host_in, non_blocking=True)
            host_out, dst = _staging(self.world * size, torch.uint8, dev, "iter_out")
            dist.all_gather_into_tensor(dst, src, group=self.group)
            if host_out is not dst:
                host_out.copy_(dst, non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
            allb = host_out.numpy().reshape(self.world, size)
            return [allb[r].copy() for r in range(self.world)]
        return [payload]

    def exchange(self, trees, scores, losses, nsub: int, counts, options, dtype):
        """Every rank's (nsub, members, counts), in rank order.  When any rank's members overflow the
        capacity (a custom complexity mapping lets trees outgrow maxsize + 1 nodes), every rank sees
        its flag in the first round and all ranks repeat the exchange once with a capacity sized from
        the largest need -- no rank raises alone while the others wait."""
        import time

        t0 = time.perf_counter()
        self.last_overflow = None
        parts = self._gather(self.pack(trees, scores, losses, nsub, counts, options, dtype))
        needs = [self.overflow(p) for p in parts]
        if any(nd is not None for nd in needs):
            own = self.needs(trees, options, dtype)
            cap = max([self.cap, own[0]] + [nd[0] for nd in needs if nd is not None])
            pool = max([self.pool, own[1]] + [nd[1] for nd in needs if nd is not None])
            wide = IterationExchange(cap, pool, self.nbin, self.comm, self.group, self.world)
            parts = wide._gather(wide.pack(trees, scores, losses, nsub, counts, options, dtype))
            self.last_overflow = (cap, pool)
            out = [wide.unpack(p, options) for p in parts]
        else:
            out = [self.unpack(p, options) for p in parts]
        timer.seconds += time.perf_counter() - t0
        timer.calls += 1
        return out

    def close(self):
        if self.comm is not None:
            self.comm.close()
            self.comm = None


class _Pending:
    """An in-flight migrate_topk exchange (migrate_topk_async): wait() -> [(nodes, offsets, losses)]."""

    def __init__(self, work, dst, host_out, ws, head, k, payload_len, t_issue):
        self.work, self.dst, self.host_out, self.ws = work, dst, host_out, ws
        self.head, self.k, self.n, self.t_issue = head, k, payload_len, t_issue

    def wait(self):
        import time

        import torch

        t0 = time.perf_counter()
        self.work.wait()
        if self.host_out is not self.dst:
            self.host_out.copy_(self.dst, non_blocking=True)
            torch.cuda.current_stream(self.dst.device).synchronize()
        allb = self.host_out.numpy().reshape(self.ws, self.n)
        out = _unpack_topk(allb, self.ws, self.head, self.k)
        timer.seconds += time.perf_counter() - t0
        timer.calls += 1
        return out


def _unpack_topk(allb, ws, head, k):
    rec = NODE_DTYPE.itemsize
    out = []
    for r in range(ws):
        h = allb[r, :head].copy().view(np.int64)
        cnt = int(h[0])
        of = h[1:cnt + 2].copy()
        ls = allb[r, 8 * (k + 2):head].copy().view(np.float64)[:cnt]
        nd = allb[r, head:head + int(of[-1]) * rec].copy().view(NODE_DTYPE)
        out.append((nd, of, ls))
    return out


def migrate_topk_async(nodes: np.ndarray, offsets: np.ndarray, losses: np.ndarray, k: int, max_nodes: int,
                       group=None) -> _Pending:
    """migrate_topk, issued and left in flight: the all-gather runs on the collective's own stream
    while the caller's next evaluation runs on the library's; .wait() collects it.  The bench issues
    step k's exchange after step k's evaluation and collects it after step k + 1's."""
    import time

    import torch

    dist = _dist()
    t0 = time.perf_counter()
    ws = dist.get_world_size(group)
    payload, head = _pack_topk(nodes, offsets, losses, k, max_nodes)
    dev = _device(group)
    host_in, src = _staging(len(payload), torch.uint8, dev, "migrate_in")
    host_in.numpy()[:] = payload
    if src is not host_in:
        src.copy_(host_in, non_blocking=True)
    host_out, dst = _staging(ws * len(payload), torch.uint8, dev, "migrate_out")
    work = dist.all_gather_into_tensor(dst, src, group=group, async_op=True)
    timer.seconds += time.perf_counter() - t0
    return _Pending(work, dst, host_out, ws, head, k, len(payload), t0)


def _pack_topk(nodes, offsets, losses, k, max_nodes):
    nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
    offsets = np.asarray(offsets, dtype=np.int64)
    losses = np.asarray(losses, dtype=np.float64)
    order = np.argsort(np.where(np.isfinite(losses), losses, np.inf), kind="stable")
    sel = [int(t) for t in order if offsets[t + 1] - offsets[t] <= max_nodes][:k]
    rec = NODE_DTYPE.itemsize
    # [count, offsets (k + 1) int64, losses k f64, nodes k * max_nodes records]
    head = 8 * (1 + (k + 1) + k)
    payload = np.zeros(head + k * max_nodes * rec, dtype=np.uint8)
    hdr = payload[:head].view(np.int64)
    hdr[0] = len(sel)
    offs_out = hdr[1:k + 2]
    loss_out = payload[8 * (k + 2):head].view(np.float64)
    cur = 0
    body = payload[head:]
    for i, t in enumerate(sel):
        a, b = int(offsets[t]), int(offsets[t + 1])
        body[cur * rec:(cur + b - a) * rec] = nodes[a:b].view(np.uint8)
        offs_out[i] = cur
        loss_out[i] = losses[t]
        cur += b - a
    offs_out[len(sel)] = cur
    return payload, head


def migrate_topk(nodes: np.ndarray, offsets: np.ndarray, losses: np.ndarray, k: int, max_nodes: int, group=None):
    """Migration exchange with a fixed-size payload: this rank's k best trees (by loss; did_succeed
    trees first) travel as node tables plus their losses in one packed buffer of
    k x max_nodes node records, so the exchange is ONE all_gather_into_tensor with no size
    round (src/Migration.jl:16-38: every population's best members reach every other).  Trees
    longer than max_nodes are skipped.  Returns [(nodes, offsets, losses)] by rank."""
    return migrate_topk_async(nodes, offsets, losses, k, max_nodes, group).wait()


def same_migrants(a, b) -> bool:
    """Two migrate_topk results ([(nodes, offsets, losses)] by rank) hold the same trees: node records
    byte for byte, offsets by value, losses bit for bit (the bench's check of the library's RCCL
    exchange against the torch.distributed one before it times the native path)."""
    if len(a) != len(b):
        return False
    for (na, oa, la), (nb, ob, lb) in zip(a, b):
        if np.ascontiguousarray(na).view(np.uint8).tobytes() != np.ascontiguousarray(nb).view(np.uint8).tobytes():
            return False
        if not np.array_equal(np.asarray(oa, np.int64), np.asarray(ob, np.int64)):
            return False
        if np.asarray(la, np.float64).tobytes() != np.asarray(lb, np.float64).tobytes():
            return False
    return True


# ---- the native exchanges: libsrhip's RCCL communicator (include/srhip.h srhip_comm_*) -----------

class _NativePending:
    """An in-flight NativeComm.migrate_start: wait() -> [(nodes, offsets, losses)] by rank."""

    def __init__(self, comm, k, max_nodes, t_issue):
        self.comm, self.k, self.max_nodes, self.t_issue = comm, k, max_nodes, t_issue

    def wait(self):
        import ctypes
        import time

        from . import _lib

        t0 = time.perf_counter()
        ws, k, mx = self.comm.nranks, self.k, self.max_nodes
        counts = np.zeros(ws, dtype=np.int32)
        offs = np.zeros((ws, k + 1), dtype=np.int64)
        losses = np.zeros((ws, k), dtype=np.float64)
        nodes = np.zeros(ws * k * mx, dtype=NODE_DTYPE)
        _lib.check(_lib.load().srhip_comm_migrate_wait(self.comm.handle, _lib.ptr(counts), _lib.ptr(offs),
                                                        _lib.ptr(losses), ctypes.c_void_p(nodes.ctypes.data)))
        out = []
        for r in range(ws):
            c = int(counts[r])
            of = offs[r, :c + 1].copy()
            nd = nodes[r * k * mx: r * k * mx + int(of[-1])].copy()
            out.append((nd, of, losses[r, :c].copy()))
        timer.seconds += time.perf_counter() - t0
        timer.calls += 1
        return out


class NativeComm:
    """libsrhip's RCCL communicator for one rank (one process per GPU): the migration all-gather and
    the row-shard all-reduces run inside the library on device buffers (csrc/srhip_comm.cpp), with no
    torch tensors on the data path.  ``from_process_group`` creates it collectively: rank 0 draws the
    communicator id and the torch.distributed group broadcasts its 128 bytes."""

    def __init__(self, ctx, nranks: int, rank: int, uid: bytes):
        import ctypes

        from . import _lib

        if len(uid) != _lib.COMM_ID_BYTES:
            raise ValueError("communicator id must be 128 bytes")
        self.ctx, self.nranks, self.rank = ctx, int(nranks), int(rank)
        self._uid = (ctypes.c_uint8 * _lib.COMM_ID_BYTES).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        _lib.check(_lib.load().srhip_comm_create(ctx.handle, ctypes.cast(self._uid, ctypes.c_void_p), self.nranks,
                                                 self.rank, ctypes.byref(h)))
        self.handle = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes

        from . import _lib

        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
        _lib.check(_lib.load().srhip_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
        return bytes(buf)

    @classmethod
    def from_process_group(cls, ctx, group=None):
        import torch

        dist = _dist()
        rank, ws = dist.get_rank(group), dist.get_world_size(group)
        uid = cls.unique_id() if rank == 0 else bytes(128)
        t = torch.tensor(list(uid), dtype=torch.uint8, device=_device(group))
        dist.broadcast(t, 0, group=group)
        return cls(ctx, ws, rank, bytes(t.cpu().numpy().tobytes()))

    def migrate_start(self, nodes, offsets, losses, k: int, max_nodes: int) -> _NativePending:
        """Issue the migration all-gather of this rank's k best trees (by loss) and return at once."""
        import ctypes
        import time

        from . import _lib

        t0 = time.perf_counter()
        nodes = np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        losses = np.ascontiguousarray(losses, dtype=np.float64)
        _lib.check(_lib.load().srhip_comm_migrate_start(self.handle, ctypes.c_void_p(nodes.ctypes.data),
                                                         _lib.ptr(offsets), len(offsets) - 1, _lib.ptr(losses),
                                                         int(k), int(max_nodes)))
        timer.seconds += time.perf_counter() - t0
        return _NativePending(self, int(k), int(max_nodes), t0)

    def migrate_topk(self, nodes, offsets, losses, k: int, max_nodes: int):
        return self.migrate_start(nodes, offsets, losses, k, max_nodes).wait()

    def allreduce_f64(self, a, op: str = "sum") -> np.ndarray:
        from . import _lib

        b = np.ascontiguousarray(a, dtype=np.float64).copy()
        _lib.check(_lib.load().srhip_comm_allreduce_f64(self.handle, _lib.ptr(b), b.size,
                                                         _lib.REDUCE_MAX if op == "max" else _lib.REDUCE_SUM))
        return b

    def allgather(self, data: bytes) -> list:
        import ctypes

        from . import _lib

        src = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        dst = np.zeros(len(src) * self.nranks, dtype=np.uint8)
        _lib.check(_lib.load().srhip_comm_allgather(self.handle, ctypes.c_void_p(src.ctypes.data), len(src),
                                                     ctypes.c_void_p(dst.ctypes.data)))
        return [dst[r * len(src):(r + 1) * len(src)].tobytes() for r in range(self.nranks)]

    def eval_loss_sharded(self, prog, ds, loss, idx=None):
        """Row-sharded eval_loss over this rank's rows (srhip_eval_loss_sharded): (loss[T], ok[T]),
        identical on every rank."""
        import ctypes
        import time

        from . import _lib

        t0 = time.perf_counter()
        out = np.empty(prog.ntrees, dtype=np.float64)
        ok = np.empty(prog.ntrees, dtype=np.uint8)
        ls = loss.c_struct()
        idxa = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
        _lib.check(_lib.load().srhip_eval_loss_sharded(self.ctx.handle, self.handle, ds.handle, prog.handle,
                                                        ctypes.byref(ls), _lib.ptr(idxa),
                                                        0 if idxa is None else len(idxa), _lib.ptr(out), _lib.ptr(ok)))
        timer.seconds += time.perf_counter() - t0
        timer.calls += 1
        return out, ok.astype(bool)

    def stats(self):
        """(ms of the last exchange, ms in all exchanges, exchanges) -- host wall time, issue to completion
        seen (srhip_comm_stats)."""
        import ctypes

        from . import _lib

        last, total, calls = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        _lib.check(_lib.load().srhip_comm_stats(self.handle, ctypes.byref(last), ctypes.byref(total),
                                                ctypes.byref(calls)))
        return last.value, total.value, calls.value

    def close(self):
        from . import _lib

        if getattr(self, "handle", None):
            _lib.load().srhip_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
