// srhip_batch.cpp — cross-population request coalescer.
//
// The reference scores a single mutated tree per call (score_func in next_generation,
// src/Mutate.jl:268-274) from every population task at once (src/SearchUtils.jl:121-122).  One
// launch per tree would leave the GPU idle between tiny kernels, so island threads submit here
// and block; worker threads turn whatever is queued into one program and one srhip_eval_loss
// launch (per distinct row subset).  Per-tree results of the interpreter do not depend on which
// other trees share the launch, so a coalesced score equals the single-tree score bit for bit.
//
// Workers (SRHIP_COALESCE_WORKERS, default 2): each owns a context (the caller's for worker 0, its
// own stream on the same device for the others) and a long-lived slot program, and takes the next
// batch when it is free -- while one worker waits for its launch, another compiles and launches
// the next batch, so host compile and device time overlap.  Each request completes through its own
// condition variable: a flush wakes exactly the clients of its batch (one shared condition woke
// every waiting client per flush: 64 native clients spent more time in wake-ups than the device
// in kernels, tools/coalescer_bench.cpp).
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "srhip_internal.h"

using namespace srhip;

namespace {

struct Result {
  int rc = SRHIP_OK;
  double loss = 0.0;
  uint8_t ok = 0;
  std::string err;
};

// one submitted request's completion: written once by a worker, read once by its waiter
struct Pending {
  std::mutex m;
  std::condition_variable cv;
  bool done = false;
  Result res;
};

struct Request {
  uint64_t ticket;
  std::vector<srhip_node> nodes;
  std::vector<int64_t> idx;
  std::chrono::steady_clock::time_point t_submit;
  std::shared_ptr<Pending> pending;
};

struct Worker {
  srhip_ctx* ctx = nullptr;   // worker 0: the caller's context; the others: owned
  bool own_ctx = false;
  srhip_program* slot = nullptr;  // the long-lived program every flush recompiles
  std::thread th;
  double busy_ms = 0.0, kernel_ms = 0.0;  // guarded by the batcher's mu
};

}  // namespace

struct srhip_batcher {
  const srhip_dataset* ds = nullptr;
  std::vector<int32_t> binops, unaops;
  srhip_loss loss{};
  int32_t max_batch = 256;
  int32_t max_wait_us = 200;
  int32_t nclients = 0;

  std::mutex mu;
  std::condition_variable cv_work;  // workers: queue changed / stop
  std::deque<Request> queue;
  std::unordered_map<uint64_t, std::shared_ptr<Pending>> pending;  // submitted, not yet waited for
  uint64_t next_ticket = 1;
  bool stop = false;
  int64_t n_requests = 0, max_seen = 0;
  std::atomic<int64_t> n_launches{0};
  std::vector<Worker> workers;
  bool w0_busy = false;  // worker 0 is inside a flush (guarded by mu)

  void run(Worker& w);
  void flush(Worker& w, std::vector<Request>& batch);
};

namespace {

// The worker's one long-lived program: every flush recompiles it in place (host) and re-uploads
// into its device buffers, which only grow -- no allocation, free or program object per flush (a
// hipFree synchronises the whole device), and the upload is not synchronised separately: the
// evaluation that follows on the same stream synchronises once, at its end.
int run_slot_program(srhip_batcher* b, Worker& w, std::vector<srhip_node>&& nodes, std::vector<int64_t>&& offs,
                     const std::vector<int64_t>& idx, double* loss, uint8_t* ok) {
  srhip_program& P = *w.slot;
  P.ntrees = (int32_t)offs.size() - 1;
  P.nodes = std::move(nodes);
  P.offsets = std::move(offs);
  int rc = compile_program(P);
  if (rc) return rc;
  rc = upload_program(P, false, true);  // uploaded with the launch's tree order, one copy
  if (rc) return rc;
  return srhip_eval_loss(w.ctx, b->ds, &P, &b->loss, idx.empty() ? nullptr : idx.data(), (int64_t)idx.size(), loss,
                         ok);
}

// One launch over the trees of `reqs` (same row subset); results in request order.
void launch_group(srhip_batcher* b, Worker& w, const std::vector<Request*>& reqs, std::vector<std::pair<Request*, Result>>& out,
                  double& kernel_ms) {
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
  int rc = run_slot_program(b, w, std::move(nodes), std::move(offs), idx, loss.data(), ok.data());
  b->n_launches++;
  if (rc == SRHIP_OK) {
    const double k = srhip_last_kernel_ms(w.ctx);
    if (k > 0.0) kernel_ms += k;
  }
  if (rc != SRHIP_OK && n > 1 && rc != SRHIP_ERR_DEVICE) {
    // a malformed / unsupported tree fails the whole program: attribute errors per request
    for (Request* r : reqs) launch_group(b, w, std::vector<Request*>{r}, out, kernel_ms);
    return;
  }
  const std::string err = rc == SRHIP_OK ? std::string() : std::string(srhip_last_error());
  for (int32_t i = 0; i < n; ++i) {
    Result res;
    res.rc = rc;
    res.loss = loss[i];
    res.ok = ok[i];
    res.err = err;
    out.emplace_back(reqs[i], std::move(res));
  }
}

}  // namespace

void srhip_batcher::flush(Worker& w, std::vector<Request>& batch) {
  const auto t0 = std::chrono::steady_clock::now();
  // group by row subset (most searches: one group, idx empty)
  std::map<std::vector<int64_t>, std::vector<Request*>> groups;
  for (Request& r : batch) groups[r.idx].push_back(&r);
  std::vector<std::pair<Request*, Result>> out;
  out.reserve(batch.size());
  double kms = 0.0;
  for (auto& g : groups) launch_group(this, w, g.second, out, kms);
  const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  {
    std::lock_guard<std::mutex> lk(mu);
    w.busy_ms += dt;
    w.kernel_ms += kms;
    n_requests += (int64_t)batch.size();
    max_seen = std::max<int64_t>(max_seen, (int64_t)batch.size());
  }
  for (auto& kv : out) {  // wake exactly this batch's clients
    Pending& pd = *kv.first->pending;
    {
      std::lock_guard<std::mutex> lk(pd.m);
      pd.res = std::move(kv.second);
      pd.done = true;
    }
    pd.cv.notify_one();
  }
}

void srhip_batcher::run(Worker& w) {
  // Worker 0 takes every batch it can; the others only while worker 0 is inside a flush (a single
  // client -- C1's latency-bound path -- then always meets worker 0 on the caller's context, and a
  // second worker adds throughput only under load)
  const bool first = &w == &workers[0];
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    cv_work.wait(lk, [&] { return stop || (!queue.empty() && (first || w0_busy)); });
    if (queue.empty() && stop) return;
    if (queue.empty()) continue;
    // gather: flush when full, when every registered client has a request queued, at the
    // deadline (clients that finished or are slow), or on stop
    const auto deadline = queue.front().t_submit + std::chrono::microseconds(max_wait_us);
    cv_work.wait_until(lk, deadline, [&] {
      return stop || queue.empty() || (int64_t)queue.size() >= max_batch ||
             (nclients > 0 && (int64_t)queue.size() >= nclients);
    });
    if (queue.empty()) continue;  // another worker took them
    std::vector<Request> batch;
    const size_t take = std::min<size_t>(queue.size(), (size_t)max_batch);
    batch.reserve(take);
    for (size_t i = 0; i < take; ++i) {
      batch.push_back(std::move(queue.front()));
      queue.pop_front();
    }
    if (first) w0_busy = true;
    if (first && !queue.empty()) cv_work.notify_all();  // the rest is for another worker
    lk.unlock();
    flush(w, batch);
    lk.lock();
    if (first) w0_busy = false;
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
  b->ds = ds;
  b->binops.assign(ops->binops, ops->binops + ops->nbin);
  b->unaops.assign(ops->unaops, ops->unaops + ops->nuna);
  if (loss) b->loss = *loss;
  b->max_batch = max_batch;
  b->max_wait_us = max_wait_us;
  static const int nworkers_env = [] { const char* e = getenv("SRHIP_COALESCE_WORKERS"); return e ? atoi(e) : 0; }();
  const int nworkers = nworkers_env >= 1 ? std::min(nworkers_env, 8) : 2;
  b->workers.resize(nworkers);
  int rc = SRHIP_OK;
  for (int i = 0; i < nworkers && rc == SRHIP_OK; ++i) {
    Worker& w = b->workers[i];
    if (i == 0) {
      w.ctx = ctx;
    } else {
      rc = srhip_ctx_create(ctx->device, &w.ctx);
      w.own_ctx = rc == SRHIP_OK;
    }
    // the slot program: an empty population for this operator table, on the worker's context
    const int64_t zero = 0;
    if (rc == SRHIP_OK) rc = srhip_program_create(w.ctx, ds->dtype, nullptr, &zero, 0, ops, &w.slot);
  }
  if (rc != SRHIP_OK) {
    for (Worker& w : b->workers) {
      srhip_program_destroy(w.slot);
      if (w.own_ctx) srhip_ctx_destroy(w.ctx);
    }
    delete b;
    return rc;
  }
  try {
    for (Worker& w : b->workers) w.th = std::thread([b, &w] { b->run(w); });
  } catch (...) {
    {
      std::lock_guard<std::mutex> lk(b->mu);
      b->stop = true;
    }
    b->cv_work.notify_all();
    for (Worker& w : b->workers)
      if (w.th.joinable()) w.th.join();
    for (Worker& w : b->workers) {
      srhip_program_destroy(w.slot);
      if (w.own_ctx) srhip_ctx_destroy(w.ctx);
    }
    delete b;
    return fail(SRHIP_ERR_NOMEM, "cannot start the batcher threads");
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
  r.pending = std::make_shared<Pending>();
  {
    std::lock_guard<std::mutex> lk(b->mu);
    if (b->stop) return fail(SRHIP_ERR_INVALID, "batcher is shutting down");
    r.ticket = b->next_ticket++;
    *ticket = r.ticket;
    b->pending.emplace(r.ticket, r.pending);
    b->queue.push_back(std::move(r));
  }
  if (b->workers.size() > 1) b->cv_work.notify_all();  // worker 0 if idle, else another
  else b->cv_work.notify_one();
  return SRHIP_OK;
}

int srhip_batcher_wait(srhip_batcher* b, uint64_t ticket, double* out_loss, uint8_t* out_ok) {
  if (!b) return fail(SRHIP_ERR_INVALID, "null batcher");
  std::shared_ptr<Pending> pd;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    auto it = b->pending.find(ticket);
    if (it == b->pending.end()) return fail(SRHIP_ERR_INVALID, "unknown ticket");
    pd = std::move(it->second);
    b->pending.erase(it);
  }
  Result res;
  {
    std::unique_lock<std::mutex> lk(pd->m);
    pd->cv.wait(lk, [&] { return pd->done; });
    res = std::move(pd->res);
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
  double bm = 0.0, km = 0.0;  // summed over the workers (busy_ms may exceed the wall time)
  for (const Worker& w : b->workers) {
    bm += w.busy_ms;
    km += w.kernel_ms;
  }
  if (busy_ms) *busy_ms = bm;
  if (kernel_ms) *kernel_ms = km;
  return SRHIP_OK;
}

void srhip_batcher_destroy(srhip_batcher* b) {
  if (!b) return;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->stop = true;
  }
  b->cv_work.notify_all();
  for (Worker& w : b->workers)
    if (w.th.joinable()) w.th.join();
  for (Worker& w : b->workers) {
    srhip_program_destroy(w.slot);
    if (w.own_ctx) srhip_ctx_destroy(w.ctx);
  }
  delete b;
}

}  // extern "C"
