// host_stress.cpp — concurrency / memory stress of libsrhip's host C++ through the C ABI, the driver the
// sanitizer builds run (SURVEY.md 5 sanitizers row; the reference's CI runs --check-bounds=yes,
// .github/workflows/CI.yml:72).  `make -C tools asan` / `make -C tools tsan` link it against a libsrhip
// whose host objects (srhip_host.cpp, srhip_batch.cpp, srhip_optim.cpp, srhip_comm.cpp) are built with
// -fsanitize=address,undefined / -fsanitize=thread (on the host side only: -Xarch_host), the sanitizer
// runtime linked into this executable -- no LD_PRELOAD.
//
// Host phase (no GPU needed): THREADS threads compile host-only programs (ctx = NULL) of random
// populations at once -- the persistent host pool, the 64-shard code cache with its first-sighting
// table (populations recur, so trees are cached on their second sighting and hit from their third),
// background teardown -- query and set constants, run srhip_partials_finalize over random partials,
// and feed malformed node tables (bad children, bad operator indices) that must fail cleanly.
// Device phase (only when a device is visible): concurrent clients of the cross-population coalescer
// (srhip_batcher: per-request completion, two worker contexts), submitted evaluations waited out of
// order (srhip_eval_loss_submit / _wait) and the split constant optimiser (three contexts and threads).
//
//   host_stress [THREADS] [ROUNDS]     prints "host_stress ok ..." and exits 0, or exits 1 on a mismatch
// On a GPU box: LSAN_OPTIONS=suppressions=tools/lsan_rocm.supp (the ROCm runtime's own allocations that
// outlive the process: libhsa-runtime64 / libamdhip64 frames only, none of libsrhip's).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../include/srhip.h"

#if defined(__has_feature)
#if __has_feature(address_sanitizer)
#define SRHIP_STRESS_ASAN 1
#include <sanitizer/lsan_interface.h>
#include <unistd.h>
#endif
#endif
#ifndef SRHIP_STRESS_ASAN
#define SRHIP_STRESS_ASAN 0
#endif

static std::atomic<int> g_fail{0};
#define CHECK(expr)                                                                           \
  do {                                                                                        \
    const int rc_ = (expr);                                                                   \
    if (rc_) {                                                                                \
      fprintf(stderr, "FAIL %s:%d %s -> %d: %s\n", __FILE__, __LINE__, #expr, rc_, srhip_last_error()); \
      g_fail = 1;                                                                             \
    }                                                                                         \
  } while (0)

static const int32_t BINOPS[] = {SRHIP_OP_ADD, SRHIP_OP_SUB, SRHIP_OP_MUL, SRHIP_OP_DIV};
static const int32_t UNAOPS[] = {SRHIP_OP_COS, SRHIP_OP_EXP};
static const srhip_operators OPS{4, 2, BINOPS, UNAOPS};

// a random tree of about `size` nodes in the node-table layout (root first, children after)
static void random_tree(std::mt19937_64& rng, int size, int nfeat, std::vector<srhip_node>& out) {
  const size_t base = out.size();
  std::vector<int> todo{0};
  out.push_back(srhip_node{});
  int budget = size - 1;
  for (size_t k = 0; k < todo.size(); ++k) {
    srhip_node& n = out[base + todo[k]];
    n.l = n.r = -1;
    const int pick = budget >= 2 ? (int)(rng() % 3) : (budget == 1 ? (int)(rng() % 2) : 0);
    if (pick == 0) {
      n.degree = 0;
      if (rng() % 2) {
        n.constant = 1;
        n.val = std::ldexp((double)(rng() % 2001) - 1000.0, -8);
      } else {
        n.constant = 0;
        n.feature = (uint16_t)(1 + rng() % nfeat);
      }
      continue;
    }
    n.degree = (uint8_t)pick;
    n.op = (uint16_t)(1 + rng() % (pick == 2 ? 4 : 2));
    const int l = (int)(out.size() - base);
    out.push_back(srhip_node{});
    out[base + todo[k]].l = l;
    todo.push_back(l);
    --budget;
    if (pick == 2) {
      const int r = (int)(out.size() - base);
      out.push_back(srhip_node{});
      out[base + todo[k]].r = r;
      todo.push_back(r);
      --budget;
    }
  }
}

struct Population {
  std::vector<srhip_node> nodes;
  std::vector<int64_t> offs{0};
};
static Population population(uint64_t seed, int ntrees, int nfeat) {
  std::mt19937_64 rng(seed);
  Population p;
  for (int t = 0; t < ntrees; ++t) {
    random_tree(rng, 1 + (int)(rng() % 30), nfeat, p.nodes);
    p.offs.push_back((int64_t)p.nodes.size());
  }
  return p;
}

static void host_worker(int id, int rounds, const std::vector<Population>* pops) {
  std::mt19937_64 rng(1000 + id);
  for (int it = 0; it < rounds; ++it) {
    const Population& p = (*pops)[(size_t)(rng() % pops->size())];
    const int32_t nt = (int32_t)p.offs.size() - 1;
    srhip_program* P = nullptr;
    CHECK(srhip_program_create(nullptr, SRHIP_F32, p.nodes.data(), p.offs.data(), nt, &OPS, &P));
    if (!P) continue;
    std::vector<int32_t> nconst(nt);
    CHECK(srhip_program_num_constants(P, nconst.data()));
    int64_t total = 0;
    for (int32_t c : nconst) total += c;
    std::vector<double> consts((size_t)total);
    CHECK(srhip_program_get_constants(P, consts.data()));
    for (double& c : consts) c *= 1.0 + 0.01 * (double)(rng() % 7);
    CHECK(srhip_program_set_constants(P, consts.data()));
    int64_t tn = 0, to = 0;
    int32_t ms = 0;
    CHECK(srhip_program_stats(P, &tn, &to, &ms));
    if (tn != p.offs.back()) {
      fprintf(stderr, "FAIL node count %lld != %lld\n", (long long)tn, (long long)p.offs.back());
      g_fail = 1;
    }
    // the row-shard decision over random partials (static-fail metadata, overflow thresholds)
    const int64_t nf = 5;
    std::vector<double> sums(2 * (size_t)nt + 2 * nf + 1), chk(nt), loss(nt);
    std::vector<uint8_t> ok(nt), status(nt);
    for (int32_t t = 0; t < nt; ++t) {
      sums[2 * t] = (double)(rng() % 1000);
      sums[2 * t + 1] = 4096.0;
      chk[t] = (rng() % 50 == 0) ? INFINITY : std::ldexp(1.0, (int)(rng() % 140));
    }
    for (int64_t f = 0; f < nf; ++f) sums[2 * (size_t)nt + 2 * f] = 1.0;
    sums[2 * (size_t)nt + 2 * nf] = 4096.0;
    CHECK(srhip_partials_finalize(P, nf, sums.data(), chk.data(), loss.data(), ok.data(), status.data()));
    srhip_program_destroy(P);  // (background teardown)
    // malformed tables: a child index past the tree, an operator index past the table
    std::vector<srhip_node> bad(p.nodes.begin(), p.nodes.begin() + p.offs[1]);
    if (!bad.empty() && bad[0].degree > 0) {
      bad[0].l = 1000;
      int64_t bo[2] = {0, (int64_t)bad.size()};
      srhip_program* Q = nullptr;
      if (srhip_program_create(nullptr, SRHIP_F32, bad.data(), bo, 1, &OPS, &Q) != SRHIP_ERR_INVALID) {
        fprintf(stderr, "FAIL malformed child index accepted\n");
        g_fail = 1;
      }
      srhip_program_destroy(Q);
      bad[0].l = p.nodes[0].l;
      bad[0].op = 99;
      if (srhip_program_create(nullptr, SRHIP_F32, bad.data(), bo, 1, &OPS, &Q) == SRHIP_OK) {
        fprintf(stderr, "FAIL malformed operator index accepted\n");
        g_fail = 1;
      }
      srhip_program_destroy(Q);
    }
  }
}

static void device_phase(int threads) {
  srhip_ctx* ctx = nullptr;
  CHECK(srhip_ctx_create(0, &ctx));
  if (!ctx) return;
  const int64_t nf = 5, n = 20000;
  std::vector<float> X((size_t)nf * n), y(n);
  std::mt19937_64 rng(7);
  std::normal_distribution<float> nd(0.0f, 1.0f);
  for (float& x : X) x = nd(rng);
  for (int64_t j = 0; j < n; ++j) y[j] = 2.0f * std::cos(X[3 * n + j]) + X[j] * X[j] - 2.0f;
  srhip_dataset* ds = nullptr;
  CHECK(srhip_dataset_create(ctx, SRHIP_F32, X.data(), nf, n, n, 1, y.data(), nullptr, &ds));
  const srhip_loss loss{SRHIP_LOSS_L2, 0, 0.0, 0.0};
  // (1) submitted evaluations, waited out of order, against srhip_eval_loss
  {
    std::vector<Population> pops;
    std::vector<srhip_program*> progs;
    for (int i = 0; i < 3; ++i) {
      pops.push_back(population(500 + i, 200, (int)nf));
      srhip_program* P = nullptr;
      CHECK(srhip_program_create(ctx, SRHIP_F32, pops[i].nodes.data(), pops[i].offs.data(), 200, &OPS, &P));
      progs.push_back(P);
    }
    std::vector<std::vector<double>> want(3, std::vector<double>(200)), got = want;
    std::vector<std::vector<uint8_t>> wok(3, std::vector<uint8_t>(200)), gok = wok;
    for (int i = 0; i < 3; ++i) CHECK(srhip_eval_loss(ctx, ds, progs[i], &loss, nullptr, 0, want[i].data(), wok[i].data()));
    srhip_eval_ticket* t[3] = {nullptr, nullptr, nullptr};
    for (int i = 0; i < 3; ++i) CHECK(srhip_eval_loss_submit(ctx, ds, progs[i], &loss, nullptr, 0, &t[i]));
    for (int i : {2, 0, 1})
      if (t[i]) CHECK(srhip_eval_loss_wait(t[i], got[i].data(), gok[i].data()));
    for (int i = 0; i < 3; ++i)
      if (memcmp(got[i].data(), want[i].data(), 200 * 8) || gok[i] != wok[i]) {
        fprintf(stderr, "FAIL submitted evaluation %d differs from srhip_eval_loss\n", i);
        g_fail = 1;
      }
    // (2) the split optimiser (three contexts / host threads)
    int64_t fc[200];
    double ol[200];
    uint8_t imp[200];
    const srhip_optim_options oo{8, 2, 11, 0.0};
    CHECK(srhip_optimize_constants(ctx, ds, progs[0], &loss, nullptr, 0, &oo, ol, imp, fc));
    for (srhip_program* P : progs) srhip_program_destroy(P);
  }
  // (3) the coalescer under concurrent clients
  {
    srhip_batcher* b = nullptr;
    CHECK(srhip_batcher_create(ctx, ds, &OPS, &loss, 64, 200, &b));
    if (b) {
      CHECK(srhip_batcher_set_clients(b, threads));
      const Population pop = population(900, 256, (int)nf);
      std::vector<std::thread> th;
      for (int c = 0; c < threads; ++c)
        th.emplace_back([&, c] {
          for (int k = 0; k < 40; ++k) {
            const int t = (c * 37 + k * 11) % 256;
            double l;
            uint8_t ok;
            CHECK(srhip_batcher_eval(b, pop.nodes.data() + pop.offs[t], pop.offs[t + 1] - pop.offs[t], nullptr, 0, &l, &ok));
          }
        });
      for (auto& x : th) x.join();
      srhip_batcher_destroy(b);
    }
  }
  srhip_dataset_destroy(ds);
  srhip_ctx_destroy(ctx);
}

int main(int argc, char** argv) {
  const int threads = argc > 1 ? atoi(argv[1]) : 6;
  const int rounds = argc > 2 ? atoi(argv[2]) : 40;
  // a few populations that recur: first sightings, cache inserts on the second, hits from the third
  std::vector<Population> pops;
  for (int i = 0; i < 6; ++i) pops.push_back(population(100 + i, 64 + 97 * i, 5));
  std::vector<std::thread> th;
  for (int i = 0; i < threads; ++i) th.emplace_back(host_worker, i, rounds, &pops);
  for (auto& t : th) t.join();
  int64_t hits = 0, misses = 0, inserts = 0;
  CHECK(srhip_code_cache_stats(&hits, &misses, &inserts));
  const bool dev = srhip_device_count() > 0;
  if (dev) device_phase(threads);
  printf("host_stress %s: %d threads x %d rounds, code cache hits %lld misses %lld inserts %lld, device phase %s\n",
         g_fail ? "FAILED" : "ok", threads, rounds, (long long)hits, (long long)misses, (long long)inserts,
         dev ? "run" : "skipped (no device)");
  fflush(stdout);  // (LeakSanitizer's report at exit ends the process with _exit: unflushed output is lost)
#if SRHIP_STRESS_ASAN
  // the leak check now, then leave without the runtime's static destructors: after a device phase the
  // HIP runtime's teardown frees memory through ASan's device allocator after it has unloaded, and
  // ASan's own CHECK aborts the process there (sanitizer_allocator_device.h, "dev_runtime_unloaded_")
  // -- not a finding in this code; the leak check above still reports any leak and fails the run
  __lsan_do_leak_check();
  fflush(stderr);
  _exit(g_fail ? 1 : 0);
#endif
  return g_fail ? 1 : 0;
}
