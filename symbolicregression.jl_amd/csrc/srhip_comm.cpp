// srhip_comm.cpp — the multi-GPU exchanges of the engine behind the C ABI, on RCCL (over xGMI on one
// MI355X node): one communicator per process and GPU, its own HIP stream, device-resident message
// buffers with pinned host staging.  Two exchanges exist:
//
//  * migration (src/Migration.jl:16-38, applied on the head node at src/SymbolicRegression.jl:933-943):
//    every rank's k best trees travel as node tables plus their losses in ONE fixed-size payload
//    [count | offsets (k + 1) | losses (k) | k x max_nodes node records], exchanged by one
//    ncclAllGather -- no size round, latency-bound on xGMI.  srhip_comm_migrate_start issues it on
//    the communicator's stream and returns (the caller's next evaluation overlaps it on the
//    context's stream); srhip_comm_migrate_wait collects it.
//  * row shards (datasets too tall for one device; the reference has no row parallelism):
//    srhip_eval_loss_sharded evaluates this rank's rows, all-reduces [sums | chk] in one device
//    buffer (sums by SUM, the check statistics by MAX for Float32 / SUM otherwise, issued as one
//    RCCL group), decides did_succeed identically on every rank, and all-reduces the precise pass's
//    per-operator sums only when some tree's overflow check is undecided.
//
// The Julia side would obtain the communicator id on rank 0 (srhip_comm_unique_id) and broadcast its
// 128 bytes with whatever launcher runs the ranks (MPI.jl, Distributed); INTEGRATION.md 6 shows the
// ccall binding.  The Python mirror (srhip/parallel.py) broadcasts it over torch.distributed.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <numeric>
#include <vector>

#include "srhip_internal.h"

using namespace srhip;

struct srhip_comm {
  srhip_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  DevBuf dsend, drecv, dred;
  HostBuf hsend, hrecv, hred;
  // the migration in flight (start -> wait)
  bool pending = false;
  // host wall time of the exchanges (issue -> completion seen), srhip_comm_stats
  double ms_last = 0.0, ms_total = 0.0;
  std::chrono::steady_clock::time_point t_issue;
  int64_t calls = 0;
  void note(std::chrono::steady_clock::time_point t0) {
    ms_last = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ms_total += ms_last;
    ++calls;
  }
  int32_t k = 0, max_nodes = 0;
  size_t payload = 0, head = 0;
};

namespace {

#define NCCL_TRY(expr)                                                                                 \
  do {                                                                                                 \
    ncclResult_t r_ = (expr);                                                                          \
    if (r_ != ncclSuccess) return fail(SRHIP_ERR_DEVICE, "%s: %s", #expr, ncclGetErrorString(r_));    \
  } while (0)

// Waits for the communicator's stream (an event recorded on it) without blocking forever: a rank that
// never joins a collective would otherwise hang every other rank inside hipStreamSynchronize.  Polls
// the event and RCCL's asynchronous error; past SRHIP_COMM_TIMEOUT_S seconds (default 300) or on an
// RCCL error the communicator is aborted (ncclCommAbort: the pending collectives are torn down) and
// every later call on it fails.  The first SRHIP_COMM_SPIN_US microseconds (default 100) spin on the
// event with no sleep -- a row-shard exchange completes in tens of microseconds, and a 20 us sleep
// granularity was a fixed cost of every step -- then the poll sleeps 20 us, 200 us after 10 ms.
int comm_wait(srhip_comm* c) {
  HIP_TRY(hipEventRecord(c->done, c->stream));
  static const double limit = [] {
    const char* e = env_get("SRHIP_COMM_TIMEOUT_S");
    const double v = e && *e ? atof(e) : 300.0;
    return v > 0 ? v : 300.0;
  }();
  static const double spin_s = [] {
    const char* e = env_get("SRHIP_COMM_SPIN_US");
    const double v = e && *e ? atof(e) : 100.0;
    return (v >= 0 ? v : 100.0) * 1e-6;
  }();
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {  // spin phase: the event only
    const hipError_t q = hipEventQuery(c->done);
    if (q == hipSuccess) return SRHIP_OK;
    if (q != hipErrorNotReady) HIP_TRY(q);
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >= spin_s) break;
    __builtin_ia32_pause();
  }
  for (unsigned it = 0;; ++it) {
    const hipError_t q = hipEventQuery(c->done);
    if (q == hipSuccess) return SRHIP_OK;
    if (q != hipErrorNotReady) HIP_TRY(q);
    ncclResult_t ae = ncclSuccess;
    if ((it & 63) == 0 && ncclCommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
      (void)ncclCommAbort(c->comm);
      c->comm = nullptr;
      return fail(SRHIP_ERR_DEVICE, "RCCL asynchronous error: %s (communicator aborted)", ncclGetErrorString(ae));
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit) {
      (void)ncclCommAbort(c->comm);
      c->comm = nullptr;
      return fail(SRHIP_ERR_DEVICE, "collective did not complete in %.0f s (a rank missing?); communicator aborted",
                  limit);
    }
    usleep(it < 500 ? 20 : 200);
  }
}

// device memory (the caller's, already complete): the collectives run on it in place, no host staging
bool is_device_ptr(const void* p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // a plain host pointer reports an error: clear it
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

#define COMM_LIVE(c) \
  do { if (!(c)->comm) return fail(SRHIP_ERR_INVALID, "communicator was aborted by an earlier error"); } while (0)

// [count int64 | offsets (k + 1) int64 | losses k f64] then k * max_nodes node records
size_t topk_head(int32_t k) { return 8 * (1 + (size_t)(k + 1) + (size_t)k); }
size_t topk_payload(int32_t k, int32_t max_nodes) {
  return topk_head(k) + (size_t)k * (size_t)max_nodes * sizeof(srhip_node);
}

// the k best trees by loss (non-finite losses rank last, ties by index), skipping trees longer than
// max_nodes, packed into dst (payload bytes)
void pack_topk(const srhip_node* nodes, const int64_t* offsets, int32_t ntrees, const double* losses, int32_t k,
               int32_t max_nodes, uint8_t* dst) {
  std::vector<int32_t> order(ntrees);
  std::iota(order.begin(), order.end(), 0);
  auto key = [&](int32_t t) { return std::isfinite(losses[t]) ? losses[t] : INFINITY; };
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return key(a) < key(b); });
  const size_t head = topk_head(k);
  memset(dst, 0, topk_payload(k, max_nodes));
  int64_t* hdr = (int64_t*)dst;
  int64_t* offs = hdr + 1;
  double* ls = (double*)(dst + 8 * (size_t)(k + 2));
  srhip_node* body = (srhip_node*)(dst + head);
  int64_t cur = 0;
  int32_t cnt = 0;
  for (int32_t t : order) {
    if (cnt == k) break;
    const int64_t a = offsets[t], b = offsets[t + 1];
    if (b - a > max_nodes) continue;
    memcpy(body + cur, nodes + a, (size_t)(b - a) * sizeof(srhip_node));
    offs[cnt] = cur;
    ls[cnt] = losses[t];
    cur += b - a;
    ++cnt;
  }
  offs[cnt] = cur;
  hdr[0] = cnt;
}

}  // namespace

extern "C" {

int srhip_comm_unique_id(uint8_t* out_id) {
  if (!out_id) return fail(SRHIP_ERR_INVALID, "null id");
  ncclUniqueId id;
  NCCL_TRY(ncclGetUniqueId(&id));
  memcpy(out_id, id.internal, NCCL_UNIQUE_ID_BYTES);
  return SRHIP_OK;
}

int srhip_comm_create(srhip_ctx* ctx, const uint8_t* id, int32_t nranks, int32_t rank, srhip_comm** out) {
  if (!ctx || !id || !out) return fail(SRHIP_ERR_INVALID, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(SRHIP_ERR_INVALID, "rank %d of %d", rank, nranks);
  *out = nullptr;
  HIP_TRY(hipSetDevice(ctx->device));
  srhip_comm* c = new srhip_comm();
  c->ctx = ctx;
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId uid;
  memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(SRHIP_ERR_DEVICE, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
    srhip_comm_destroy(c);
    return fail(SRHIP_ERR_DEVICE, "comm stream / event creation failed");
  }
  *out = c;
  return SRHIP_OK;
}

void srhip_comm_destroy(srhip_comm* c) {
  if (!c) return;
  (void)hipSetDevice(c->ctx->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);  // (an aborted communicator is already gone)
  if (c->done) (void)hipEventDestroy(c->done);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int srhip_comm_stats(const srhip_comm* c, double* ms_last, double* ms_total, int64_t* calls) {
  if (!c) return fail(SRHIP_ERR_INVALID, "null communicator");
  if (ms_last) *ms_last = c->ms_last;
  if (ms_total) *ms_total = c->ms_total;
  if (calls) *calls = c->calls;
  return SRHIP_OK;
}

int srhip_comm_size(const srhip_comm* c, int32_t* nranks, int32_t* rank) {
  if (!c) return fail(SRHIP_ERR_INVALID, "null communicator");
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank;
  return SRHIP_OK;
}

int srhip_comm_allreduce_f64(srhip_comm* c, double* buf, int64_t n, int32_t op) {
  if (!c || (!buf && n > 0) || n < 0) return fail(SRHIP_ERR_INVALID, "null argument");
  COMM_LIVE(c);
  if (op != SRHIP_REDUCE_SUM && op != SRHIP_REDUCE_MAX) return fail(SRHIP_ERR_INVALID, "reduce op %d", op);
  if (c->pending) return fail(SRHIP_ERR_INVALID, "a migration is in flight on this communicator");
  if (n == 0) return SRHIP_OK;
  HIP_TRY(hipSetDevice(c->ctx->device));
  const size_t bytes = (size_t)n * 8;
  const auto t0 = std::chrono::steady_clock::now();
  if (is_device_ptr(buf)) {  // in place on the caller's device buffer
    NCCL_TRY(ncclAllReduce(buf, buf, (size_t)n, ncclFloat64, op == SRHIP_REDUCE_MAX ? ncclMax : ncclSum, c->comm,
                           c->stream));
    const int rc = comm_wait(c);
    if (rc) return rc;
    c->note(t0);
    return SRHIP_OK;
  }
  HIP_TRY(c->hred.ensure(bytes));
  HIP_TRY(c->dred.ensure(bytes));
  memcpy(c->hred.p, buf, bytes);
  HIP_TRY(hipMemcpyAsync(c->dred.p, c->hred.p, bytes, hipMemcpyHostToDevice, c->stream));
  NCCL_TRY(ncclAllReduce(c->dred.p, c->dred.p, (size_t)n, ncclFloat64, op == SRHIP_REDUCE_MAX ? ncclMax : ncclSum,
                         c->comm, c->stream));
  HIP_TRY(hipMemcpyAsync(c->hred.p, c->dred.p, bytes, hipMemcpyDeviceToHost, c->stream));
  const int rc = comm_wait(c);
  if (rc) return rc;
  memcpy(buf, c->hred.p, bytes);
  c->note(t0);
  return SRHIP_OK;
}

int srhip_comm_allgather(srhip_comm* c, const void* send, int64_t bytes, void* recv) {
  if (!c || bytes < 0 || (bytes > 0 && (!send || !recv))) return fail(SRHIP_ERR_INVALID, "null argument");
  COMM_LIVE(c);
  if (c->pending) return fail(SRHIP_ERR_INVALID, "a migration is in flight on this communicator");
  if (bytes == 0) return SRHIP_OK;
  HIP_TRY(hipSetDevice(c->ctx->device));
  const size_t b = (size_t)bytes, all = b * (size_t)c->nranks;
  const auto t0 = std::chrono::steady_clock::now();
  if (is_device_ptr(send) && is_device_ptr(recv)) {  // device to device, no staging
    NCCL_TRY(ncclAllGather(send, recv, b, ncclUint8, c->comm, c->stream));
    const int rc = comm_wait(c);
    if (rc) return rc;
    c->note(t0);
    return SRHIP_OK;
  }
  HIP_TRY(c->hsend.ensure(b));
  HIP_TRY(c->dsend.ensure(b));
  HIP_TRY(c->hrecv.ensure(all));
  HIP_TRY(c->drecv.ensure(all));
  memcpy(c->hsend.p, send, b);
  HIP_TRY(hipMemcpyAsync(c->dsend.p, c->hsend.p, b, hipMemcpyHostToDevice, c->stream));
  NCCL_TRY(ncclAllGather(c->dsend.p, c->drecv.p, b, ncclUint8, c->comm, c->stream));
  HIP_TRY(hipMemcpyAsync(c->hrecv.p, c->drecv.p, all, hipMemcpyDeviceToHost, c->stream));
  const int rc = comm_wait(c);
  if (rc) return rc;
  memcpy(recv, c->hrecv.p, all);
  c->note(t0);
  return SRHIP_OK;
}

int srhip_comm_migrate_start(srhip_comm* c, const srhip_node* nodes, const int64_t* offsets, int32_t ntrees,
                             const double* losses, int32_t k, int32_t max_nodes) {
  if (!c || !offsets || (ntrees > 0 && (!nodes || !losses)) || ntrees < 0 || k < 1 || max_nodes < 1)
    return fail(SRHIP_ERR_INVALID, "invalid argument");
  if (c->pending) return fail(SRHIP_ERR_INVALID, "a migration is already in flight on this communicator");
  COMM_LIVE(c);
  for (int32_t t = 0; t < ntrees; ++t)
    if (offsets[t + 1] < offsets[t]) return fail(SRHIP_ERR_INVALID, "offsets not ascending at tree %d", t);
  HIP_TRY(hipSetDevice(c->ctx->device));
  const auto t_issue = std::chrono::steady_clock::now();
  const size_t pl = topk_payload(k, max_nodes), all = pl * (size_t)c->nranks;
  HIP_TRY(c->hsend.ensure(pl));
  HIP_TRY(c->dsend.ensure(pl));
  HIP_TRY(c->hrecv.ensure(all));
  HIP_TRY(c->drecv.ensure(all));
  pack_topk(nodes, offsets, ntrees, losses, k, max_nodes, (uint8_t*)c->hsend.p);
  HIP_TRY(hipMemcpyAsync(c->dsend.p, c->hsend.p, pl, hipMemcpyHostToDevice, c->stream));
  NCCL_TRY(ncclAllGather(c->dsend.p, c->drecv.p, pl, ncclUint8, c->comm, c->stream));
  HIP_TRY(hipMemcpyAsync(c->hrecv.p, c->drecv.p, all, hipMemcpyDeviceToHost, c->stream));
  c->pending = true;
  c->t_issue = t_issue;
  c->k = k;
  c->max_nodes = max_nodes;
  c->payload = pl;
  c->head = topk_head(k);
  return SRHIP_OK;
}

int srhip_comm_migrate_wait(srhip_comm* c, int32_t* out_counts, int64_t* out_offsets, double* out_losses,
                            srhip_node* out_nodes) {
  if (!c) return fail(SRHIP_ERR_INVALID, "null communicator");
  if (!c->pending) return fail(SRHIP_ERR_INVALID, "no migration in flight");
  c->pending = false;
  HIP_TRY(hipSetDevice(c->ctx->device));
  {
    const int rc = comm_wait(c);
    if (rc) return rc;
  }
  c->note(c->t_issue);  // (issue -> collected: includes the caller's work in between)
  const int32_t k = c->k, mx = c->max_nodes;
  for (int r = 0; r < c->nranks; ++r) {
    const uint8_t* src = (const uint8_t*)c->hrecv.p + (size_t)r * c->payload;
    const int64_t* hdr = (const int64_t*)src;
    const int32_t cnt = (int32_t)std::min<int64_t>(std::max<int64_t>(hdr[0], 0), k);
    if (out_counts) out_counts[r] = cnt;
    if (out_offsets)
      for (int32_t i = 0; i <= k; ++i) out_offsets[(size_t)r * (k + 1) + i] = i <= cnt ? hdr[1 + i] : hdr[1 + cnt];
    if (out_losses) memcpy(out_losses + (size_t)r * k, src + 8 * (size_t)(k + 2), (size_t)k * 8);
    if (out_nodes)
      memcpy(out_nodes + (size_t)r * k * mx, src + c->head, (size_t)k * mx * sizeof(srhip_node));
  }
  return SRHIP_OK;
}

int srhip_eval_loss_sharded(srhip_ctx* ctx, srhip_comm* c, const srhip_dataset* ds, const srhip_program* P,
                            const srhip_loss* loss, const int64_t* idx, int64_t nidx, double* out_loss,
                            uint8_t* out_ok) {
  if (!c) return fail(SRHIP_ERR_INVALID, "null communicator");
  if (c->pending) return fail(SRHIP_ERR_INVALID, "a migration is in flight on this communicator");
  COMM_LIVE(c);
  if (ctx && c->ctx->device != ctx->device) return fail(SRHIP_ERR_INVALID, "communicator is on another device");
  // the partials never leave the device before they are reduced: the evaluation's reduction kernel writes
  // [loss | chk] into the communicator's device buffer, the host adds only the few aux values behind
  // them, and one RCCL group reduces the three segments in place on the communicator's stream (the
  // evaluation has completed: run_eval_sharded synchronised its stream before calling reduce)
  ShardIO io;
  io.buffer = [c](size_t bytes, void** d) -> int {
    HIP_TRY(c->dred.ensure(bytes));
    *d = c->dred.p;
    return SRHIP_OK;
  };
  io.reduce = [c](const ShardLayout& L, const double* aux, const void** out) -> int {
    const auto t0 = std::chrono::steady_clock::now();
    const size_t bytes = L.bytes();
    HIP_TRY(c->hred.ensure(bytes));
    uint8_t* h = (uint8_t*)c->hred.p;
    uint8_t* d = (uint8_t*)c->dred.p;
    memcpy(h + L.aux_off(), aux, L.naux * 8);
    HIP_TRY(hipMemcpyAsync(d + L.aux_off(), h + L.aux_off(), L.naux * 8, hipMemcpyHostToDevice, c->stream));
    NCCL_TRY(ncclGroupStart());
    ncclResult_t r1 = ncclSuccess, r2 = ncclSuccess, r3 = ncclSuccess;
    r1 = ncclAllReduce(d, d, L.nt, L.dtype == SRHIP_I32 ? ncclInt64 : ncclFloat64, ncclSum, c->comm, c->stream);
    if (r1 == ncclSuccess && L.chk_size())
      r2 = ncclAllReduce(d + L.chk_off(), d + L.chk_off(), L.nt, L.dtype == SRHIP_F32 ? ncclFloat32 : ncclFloat64,
                         L.dtype == SRHIP_F32 ? ncclMax : ncclSum, c->comm, c->stream);
    if (r1 == ncclSuccess && r2 == ncclSuccess)
      r3 = ncclAllReduce(d + L.aux_off(), d + L.aux_off(), L.naux, ncclFloat64, ncclSum, c->comm, c->stream);
    const ncclResult_t r4 = ncclGroupEnd();  // closed on every path
    NCCL_TRY(r1);
    NCCL_TRY(r2);
    NCCL_TRY(r3);
    NCCL_TRY(r4);
    HIP_TRY(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, c->stream));
    const int rc = comm_wait(c);
    if (rc) return rc;
    *out = h;
    c->note(t0);
    return SRHIP_OK;
  };
  io.reduce_host = [c](double* buf, size_t n) -> int {
    if (n == 0) return SRHIP_OK;
    const auto t0 = std::chrono::steady_clock::now();
    const size_t bytes = n * 8;
    HIP_TRY(c->hred.ensure(bytes));
    HIP_TRY(c->dred.ensure(bytes));
    memcpy(c->hred.p, buf, bytes);
    HIP_TRY(hipMemcpyAsync(c->dred.p, c->hred.p, bytes, hipMemcpyHostToDevice, c->stream));
    NCCL_TRY(ncclAllReduce(c->dred.p, c->dred.p, n, ncclFloat64, ncclSum, c->comm, c->stream));
    HIP_TRY(hipMemcpyAsync(c->hred.p, c->dred.p, bytes, hipMemcpyDeviceToHost, c->stream));
    const int rc = comm_wait(c);
    if (rc) return rc;
    memcpy(buf, c->hred.p, bytes);
    c->note(t0);
    return SRHIP_OK;
  };
  return run_eval_sharded(ctx, ds, P, loss, idx, nidx, io, out_loss, out_ok);
}

}  // extern "C"
