// coalescer_bench.cpp — the cross-population coalescer (srhip_batcher) driven by
// native client threads through the C ABI, without the Python search harness's GIL: every client
// submits one tree at a time (srhip_batcher_eval, as an island thread scores a mutation) for a fixed
// wall time, and the driver reports requests/s, node-row evals/s, the average batch per device
// launch and the device-busy fraction.  A one-thread srhip_eval_loss loop over single-tree programs
// (no coalescer) is timed beside it.
//
//   coalescer_bench DIR NCLIENTS SECONDS [MAX_BATCH] [MAX_WAIT_US]
// DIR holds meta.txt ("dtype nfeat n ntrees nbin nuna" then the bin and una op codes), nodes.bin
// (srhip_node records), offs.bin (int64 ntrees + 1), X.bin ([nfeat][n]) and y.bin, written by
// scripts/coalescer_native.py.  Prints one JSON line.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../include/srhip.h"

#define CHECK(expr)                                                                  \
  do {                                                                               \
    int rc_ = (expr);                                                                \
    if (rc_) {                                                                       \
      fprintf(stderr, "FAIL %s -> %d: %s\n", #expr, rc_, srhip_last_error());        \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)

template <typename T> static std::vector<T> load(const std::string& path) {
  std::ifstream f(path, std::ios::binary | std::ios::ate);
  if (!f) {
    fprintf(stderr, "cannot open %s\n", path.c_str());
    exit(2);
  }
  const size_t bytes = (size_t)f.tellg();
  std::vector<T> v(bytes / sizeof(T));
  f.seekg(0);
  f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)bytes);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s DIR NCLIENTS SECONDS [MAX_BATCH] [MAX_WAIT_US]\n", argv[0]);
    return 2;
  }
  const std::string dir = argv[1];
  const int nclients = atoi(argv[2]);
  const double seconds = atof(argv[3]);
  const int max_batch = argc > 4 ? atoi(argv[4]) : 256;
  const int max_wait_us = argc > 5 ? atoi(argv[5]) : 0;
  std::ifstream meta(dir + "/meta.txt");
  int dtype, nbin, nuna;
  int64_t nfeat, n, ntrees;
  meta >> dtype >> nfeat >> n >> ntrees >> nbin >> nuna;
  std::vector<int32_t> binops(nbin), unaops(nuna);
  for (auto& b : binops) meta >> b;
  for (auto& u : unaops) meta >> u;
  const auto nodes = load<srhip_node>(dir + "/nodes.bin");
  const auto offs = load<int64_t>(dir + "/offs.bin");
  const auto X = load<unsigned char>(dir + "/X.bin");
  const auto y = load<unsigned char>(dir + "/y.bin");

  srhip_ctx* ctx;
  CHECK(srhip_ctx_create(0, &ctx));
  srhip_dataset* ds;
  CHECK(srhip_dataset_create(ctx, dtype, X.data(), nfeat, n, n, 1, y.data(), nullptr, &ds));
  srhip_operators ops{nbin, nuna, binops.data(), unaops.data()};
  srhip_loss loss{SRHIP_LOSS_L2, 0, 0.0, 0.0};

  // (1) no coalescer: one thread, a fresh single-tree program per request
  auto t0 = std::chrono::steady_clock::now();
  int64_t direct = 0, direct_nodes = 0;
  for (;; ++direct) {
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > seconds / 4) break;
    const int64_t t = direct % ntrees;
    const int64_t o[2] = {0, offs[t + 1] - offs[t]};
    srhip_program* p;
    CHECK(srhip_program_create(ctx, dtype, nodes.data() + offs[t], o, 1, &ops, &p));
    double l;
    uint8_t ok;
    CHECK(srhip_eval_loss(ctx, ds, p, &loss, nullptr, 0, &l, &ok));
    srhip_program_destroy(p);
    direct_nodes += o[1];
  }
  const double direct_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

  // (2) the coalescer with NCLIENTS concurrent native clients
  srhip_batcher* b;
  CHECK(srhip_batcher_create(ctx, ds, &ops, &loss, max_batch, max_wait_us, &b));
  CHECK(srhip_batcher_set_clients(b, nclients));
  std::atomic<int64_t> served{0}, node_count{0};
  std::atomic<bool> go{false};
  std::vector<std::thread> th;
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds + 0.5);
  for (int c = 0; c < nclients; ++c)
    th.emplace_back([&, c] {
      while (!go.load()) std::this_thread::yield();
      for (int64_t k = 0; std::chrono::steady_clock::now() < deadline; ++k) {
        const int64_t t = (c + k * nclients) % ntrees;
        double l;
        uint8_t ok;
        CHECK(srhip_batcher_eval(b, nodes.data() + offs[t], offs[t + 1] - offs[t], nullptr, 0, &l, &ok));
        served++;
        node_count += offs[t + 1] - offs[t];
      }
    });
  t0 = std::chrono::steady_clock::now();
  go = true;
  for (auto& t : th) t.join();
  const double wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  int64_t nreq, nlaunch, maxb;
  double busy_ms, kernel_ms;
  CHECK(srhip_batcher_stats(b, &nreq, &nlaunch, &maxb));
  CHECK(srhip_batcher_timing(b, &busy_ms, &kernel_ms));
  srhip_batcher_destroy(b);
  printf("{\"clients\": %d, \"rows\": %lld, \"trees_in_pool\": %lld, \"wall_s\": %.3f, \"requests\": %lld, "
         "\"launches\": %lld, \"avg_batch\": %.2f, \"max_batch\": %lld, \"requests_per_s\": %.1f, "
         "\"node_rows_per_s\": %.4g, \"device_busy_frac\": %.3f, \"worker_busy_frac\": %.3f, "
         "\"no_coalescer\": {\"requests_per_s\": %.1f, \"node_rows_per_s\": %.4g}}\n",
         nclients, (long long)n, (long long)ntrees, wall, (long long)nreq, (long long)nlaunch,
         nlaunch ? (double)nreq / nlaunch : 0.0, (long long)maxb, served.load() / wall,
         (double)node_count.load() * n / wall, kernel_ms / (wall * 1e3), busy_ms / (wall * 1e3), direct / direct_s,
         (double)direct_nodes * n / direct_s);
  srhip_dataset_destroy(ds);
  srhip_ctx_destroy(ctx);
  return 0;
}
