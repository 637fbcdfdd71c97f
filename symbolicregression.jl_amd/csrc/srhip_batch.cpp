// srhip_batch.cpp — cross-population request coalescer.
//
// The reference scores a single mutated tree per call (score_func in next_generation,
// src/Mutate.jl:268-274) from every population task at once (src/SearchUtils.jl:121-122).  One
// launch per tree would leave the GPU idle between tiny kernels, so island threads submit here
// and block; a single worker thread owns the context and turns whatever is queued into one
// program and one srhip_eval_loss launch (per distinct row subset).  Per-tree results of the
// interpreter do not depend on which other trees share the launch, so a coalesced score equals
// the single-tree score bit for bit.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "srhip_internal.h"

using namespace srhip;

namespace {

struct Request {
  uint64_t ticket;
  std::vector<srhip_node> nodes;
  std::vector<int64_t> idx;
  std::chrono::steady_clock::time_point t_submit;
};

struct Result {
  int rc = SRHIP_OK;
  double loss = 0.0;
  uint8_t ok = 0;
  std::string err;
};

}  // namespace

struct srhip_batcher {
  srhip_ctx* ctx = nullptr;
  const srhip_dataset* ds = nullptr;
  std::vector<int32_t> binops, unaops;
  srhip_loss loss{};
  int32_t max_batch = 256;
  int32_t max_wait_us = 200;
  int32_t nclients = 0;

  std::mutex mu;
  std::condition_variable cv_work;  // worker: queue changed / stop
  std::condition_variable cv_done;  // clients: results posted
  std::deque<Request> queue;
  std::unordered_map<uint64_t, Result> results;
  uint64_t next_ticket = 1;
  bool stop = false;
  int64_t n_requests = 0, max_seen = 0;
  std::atomic<int64_t> n_launches{0};
  double busy_ms = 0.0, kernel_ms = 0.0;  // worker: wall time inside flushes, interpreter time (HIP events)
  std::thread worker;
  srhip_program* slot = nullptr;  // the long-lived program every flush recompiles (worker thread only)

  void run();
  void flush(std::vector<Request>& batch);
};

namespace {

// The batcher's one long-lived program: every flush recompiles it in place (host) and re-uploads
// into its device buffers, which only grow -- no allocation, free or program object per flush (a
// hipFree synchronises the whole device), and the upload is not synchronised separately: the
// evaluation that follows on the same stream synchronises once, at its end.
int run_slot_program(srhip_batcher* b, std::vector<srhip_node>&& nodes, std::vector<int64_t>&& offs,
                     const std::vector<int64_t>& idx, double* loss, uint8_t* ok) {
  srhip_program& P = *b->slot;
  P.ntrees = (int32_t)offs.size() - 1;
  P.nodes = std::move(nodes);
  P.offsets = std::move(offs);
  int rc = compile_program(P);
  if (rc) return rc;
  rc = upload_program(P, false, true);  // uploaded with the launch's tree order, one copy
  if (rc) return rc;
  return srhip_eval_loss(b->ctx, b->ds, &P, &b->loss, idx.empty() ? nullptr : idx.data(), (int64_t)idx.size(), loss, ok);
}

// One launch over the trees of `reqs` (same row subset); results keyed by ticket.
void launch_group(srhip_batcher* b, const std::vector<Request*>& reqs, std::vector<std::pair<uint64_t, Result>>& out) {
  const int32_t n = (int32_t)reqs.size();
  std::vector<srhip_node> nodes;
  std::vector<int64_t> offs(1, 0);
  for (const Request* r : reqs) {
    nodes.insert(nodes.end(), r->nodes.begin(), r->nodes.end());
    offs.push_back((int64_t)nodes.size());
  }
  const std::vector<int64_t>& idx = reqs[0]->idx;
  std::vector<double> loss(n);
  std::vector<uint8_t> ok(n);
  int rc = run_slot_program(b, std::move(nodes), std::move(offs), idx, loss.data(), ok.data());
  b->n_launches++;
  if (rc == SRHIP_OK) {
    const double k = srhip_last_kernel_ms(b->ctx);
    if (k > 0.0) b->kernel_ms += k;  // written by the worker thread only, read under mu after flush
  }
  if (rc != SRHIP_OK && n > 1 && rc != SRHIP_ERR_DEVICE) {
    // a malformed / unsupported tree fails the whole program: attribute errors per request
    for (const Request* r : reqs) launch_group(b, std::vector<Request*>{const_cast<Request*>(r)}, out);
    return;
  }
  const std::string err = rc == SRHIP_OK ? std::string() : std::string(srhip_last_error());
  for (int32_t i = 0; i < n; ++i) {
    Result res;
    res.rc = rc;
    res.loss = loss[i];
    res.ok = ok[i];
    res.err = err;
    out.emplace_back(reqs[i]->ticket, std::move(res));
  }
}

}  // namespace

void srhip_batcher::flush(std::vector<Request>& batch) {
  const auto t0 = std::chrono::steady_clock::now();
  // group by row subset (most searches: one group, idx empty)
  std::map<std::vector<int64_t>, std::vector<Request*>> groups;
  for (Request& r : batch) groups[r.idx].push_back(&r);
  std::vector<std::pair<uint64_t, Result>> out;
  out.reserve(batch.size());
  for (auto& g : groups) launch_group(this, g.second, out);
  const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  {
    std::lock_guard<std::mutex> lk(mu);
    busy_ms += dt;
    for (auto& kv : out) results[kv.first] = std::move(kv.second);
    n_requests += (int64_t)batch.size();
    max_seen = std::max<int64_t>(max_seen, (int64_t)batch.size());
  }
  cv_done.notify_all();
}

void srhip_batcher::run() {
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    cv_work.wait(lk, [&] { return stop || !queue.empty(); });
    if (queue.empty() && stop) return;
    // gather: flush when full, when every registered client has a request queued, at the
    // deadline (clients that finished or are slow), or on stop
    const auto deadline = queue.front().t_submit + std::chrono::microseconds(max_wait_us);
    cv_work.wait_until(lk, deadline, [&] {
      return stop || (int64_t)queue.size() >= max_batch || (nclients > 0 && (int64_t)queue.size() >= nclients);
    });
    std::vector<Request> batch;
    const size_t take = std::min<size_t>(queue.size(), (size_t)max_batch);
    batch.reserve(take);
    for (size_t i = 0; i < take; ++i) {
      batch.push_back(std::move(queue.front()));
      queue.pop_front();
    }
    lk.unlock();
    flush(batch);
    lk.lock();
  }
}

extern "C" {

int srhip_batcher_create(srhip_ctx* ctx, const srhip_dataset* ds, const srhip_operators* ops, const srhip_loss* loss,
                         int32_t max_batch, int32_t max_wait_us, srhip_batcher** out) {
  if (!ctx || !ds || !ops || !out) return fail(SRHIP_ERR_INVALID, "null argument");
  if (max_batch < 1 || max_wait_us < 0) return fail(SRHIP_ERR_INVALID, "max_batch >= 1 and max_wait_us >= 0 required");
  if ((ops->nbin > 0 && !ops->binops) || (ops->nuna > 0 && !ops->unaops) || ops->nbin < 0 || ops->nuna < 0)
    return fail(SRHIP_ERR_INVALID, "malformed operator table");
  srhip_batcher* b = new (std::nothrow) srhip_batcher();
  if (!b) return fail(SRHIP_ERR_NOMEM, "batcher allocation");
  b->ctx = ctx;
  b->ds = ds;
  b->binops.assign(ops->binops, ops->binops + ops->nbin);
  b->unaops.assign(ops->unaops, ops->unaops + ops->nuna);
  if (loss) b->loss = *loss;
  b->max_batch = max_batch;
  b->max_wait_us = max_wait_us;
  // the slot program: an empty population for this operator table, on the batcher's context
  const int64_t zero = 0;
  int rc = srhip_program_create(ctx, ds->dtype, nullptr, &zero, 0, ops, &b->slot);
  if (rc) {
    delete b;
    return rc;
  }
  try {
    b->worker = std::thread([b] { b->run(); });
  } catch (...) {
    delete b;
    return fail(SRHIP_ERR_NOMEM, "cannot start the batcher thread");
  }
  *out = b;
  return SRHIP_OK;
}

int srhip_batcher_set_clients(srhip_batcher* b, int32_t nclients) {
  if (!b || nclients < 0) return fail(SRHIP_ERR_INVALID, "bad batcher / client count");
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->nclients = nclients;
  }
  b->cv_work.notify_all();
  return SRHIP_OK;
}

int srhip_batcher_submit(srhip_batcher* b, const srhip_node* nodes, int64_t nnodes, const int64_t* idx, int64_t nidx,
                         uint64_t* ticket) {
  if (!b || !nodes || nnodes < 1 || !ticket) return fail(SRHIP_ERR_INVALID, "bad submit arguments");
  if (nidx < 0 || (nidx > 0 && !idx)) return fail(SRHIP_ERR_INVALID, "bad row subset");
  Request r;
  r.nodes.assign(nodes, nodes + nnodes);
  if (nidx > 0) r.idx.assign(idx, idx + nidx);
  r.t_submit = std::chrono::steady_clock::now();
  {
    std::lock_guard<std::mutex> lk(b->mu);
    if (b->stop) return fail(SRHIP_ERR_INVALID, "batcher is shutting down");
    r.ticket = b->next_ticket++;
    *ticket = r.ticket;
    b->queue.push_back(std::move(r));
  }
  b->cv_work.notify_one();
  return SRHIP_OK;
}

int srhip_batcher_wait(srhip_batcher* b, uint64_t ticket, double* out_loss, uint8_t* out_ok) {
  if (!b) return fail(SRHIP_ERR_INVALID, "null batcher");
  Result res;
  {
    std::unique_lock<std::mutex> lk(b->mu);
    if (ticket == 0 || ticket >= b->next_ticket) return fail(SRHIP_ERR_INVALID, "unknown ticket");
    b->cv_done.wait(lk, [&] { return b->results.count(ticket) != 0; });
    auto it = b->results.find(ticket);
    res = std::move(it->second);
    b->results.erase(it);
  }
  if (res.rc != SRHIP_OK) return fail(res.rc, res.err.c_str());
  if (out_loss) *out_loss = res.loss;
  if (out_ok) *out_ok = res.ok;
  return SRHIP_OK;
}

int srhip_batcher_eval(srhip_batcher* b, const srhip_node* nodes, int64_t nnodes, const int64_t* idx, int64_t nidx,
                       double* out_loss, uint8_t* out_ok) {
  uint64_t t = 0;
  int rc = srhip_batcher_submit(b, nodes, nnodes, idx, nidx, &t);
  if (rc) return rc;
  return srhip_batcher_wait(b, t, out_loss, out_ok);
}

int srhip_batcher_stats(const srhip_batcher* b, int64_t* nrequests, int64_t* nlaunches, int64_t* max_batch_seen) {
  if (!b) return fail(SRHIP_ERR_INVALID, "null batcher");
  std::lock_guard<std::mutex> lk(const_cast<srhip_batcher*>(b)->mu);
  if (nrequests) *nrequests = b->n_requests;
  if (nlaunches) *nlaunches = b->n_launches.load();
  if (max_batch_seen) *max_batch_seen = b->max_seen;
  return SRHIP_OK;
}

int srhip_batcher_timing(const srhip_batcher* b, double* busy_ms, double* kernel_ms) {
  if (!b) return fail(SRHIP_ERR_INVALID, "null batcher");
  std::lock_guard<std::mutex> lk(const_cast<srhip_batcher*>(b)->mu);
  if (busy_ms) *busy_ms = b->busy_ms;
  if (kernel_ms) *kernel_ms = b->kernel_ms;
  return SRHIP_OK;
}

void srhip_batcher_destroy(srhip_batcher* b) {
  if (!b) return;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->stop = true;
  }
  b->cv_work.notify_all();
  if (b->worker.joinable()) b->worker.join();
  srhip_program_destroy(b->slot);
  delete b;
}

}  // extern "C"
