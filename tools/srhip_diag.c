/* srhip_diag.c — step-by-step smoke of libsrhip.so through the C ABI, one flushed line per step,
 * so that a GPU hang or fault names the call it happened in.  Not a test: tests/ hold the parity
 * checks.  Build: make -C tools ; run: tools/build/srhip_diag [path/to/libsrhip.so]  */
#include <dlfcn.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/srhip.h"

#define STEP(...) do { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); fflush(stderr); } while (0)
#define CHECK(expr) do { int rc_ = (expr); if (rc_) { STEP("FAIL %s -> %d: %s", #expr, rc_, srhip_last_error()); exit(2); } } while (0)

static srhip_node leaf_f(int f) { srhip_node n; memset(&n, 0, sizeof n); n.feature = (uint16_t)f; n.l = n.r = -1; return n; }
static srhip_node leaf_c(double v) { srhip_node n; memset(&n, 0, sizeof n); n.constant = 1; n.val = v; n.l = n.r = -1; return n; }
static srhip_node un(int op, int l) { srhip_node n; memset(&n, 0, sizeof n); n.degree = 1; n.op = (uint16_t)op; n.l = l; n.r = -1; return n; }
static srhip_node bin(int op, int l, int r) { srhip_node n; memset(&n, 0, sizeof n); n.degree = 2; n.op = (uint16_t)op; n.l = l; n.r = r; return n; }

int main(void) {
  STEP("version %s, devices %d", srhip_version(), srhip_device_count());
  srhip_ctx* ctx;
  CHECK(srhip_ctx_create(0, &ctx));
  STEP("ctx ok");
  enum { NF = 3, N = 100 };
  float X[NF * N], y[N];
  for (int j = 0; j < N; ++j) {
    for (int f = 0; f < NF; ++f) X[f * N + j] = (float)sin(0.37 * j + f);
    y[j] = 2.0f * X[0 * N + j];
  }
  srhip_dataset* ds;
  CHECK(srhip_dataset_create(ctx, SRHIP_F32, X, NF, N, N, 1, y, NULL, &ds));
  STEP("dataset ok");
  int32_t binops[4] = {SRHIP_OP_ADD, SRHIP_OP_SUB, SRHIP_OP_MUL, SRHIP_OP_DIV};
  int32_t unaops[2] = {SRHIP_OP_COS, SRHIP_OP_EXP};
  srhip_operators ops = {4, 2, binops, unaops};
  /* trees: x1 | x1 + x2 | cos(x1) | (x1 * 2.0) - cos(x2 / x3) */
  srhip_node nodes[32];
  int64_t off[5];
  int k = 0;
  off[0] = k; nodes[k++] = leaf_f(1);
  off[1] = k; nodes[k++] = bin(1, 1, 2); nodes[k++] = leaf_f(1); nodes[k++] = leaf_f(2);
  off[2] = k; nodes[k++] = un(1, 1); nodes[k++] = leaf_f(1);
  off[3] = k; nodes[k++] = bin(2, 1, 4); nodes[k++] = bin(3, 2, 3); nodes[k++] = leaf_f(1); nodes[k++] = leaf_c(2.0);
  nodes[k++] = un(1, 5); nodes[k++] = bin(4, 6, 7); nodes[k++] = leaf_f(2); nodes[k++] = leaf_f(3);
  off[4] = k;
  for (int t = 0; t < 4; ++t) {
    srhip_program* P;
    int64_t o1[2] = {0, off[t + 1] - off[t]};
    CHECK(srhip_program_create(ctx, SRHIP_F32, nodes + off[t], o1, 1, &ops, &P));
    STEP("tree %d: program ok", t);
    float pred[N];
    uint8_t ok;
    CHECK(srhip_eval_predict(ctx, ds, P, NULL, 0, pred, &ok));
    STEP("tree %d: predict ok=%d pred[0..2]=%g %g %g (%.3f ms)", t, ok, pred[0], pred[1], pred[2], srhip_last_kernel_ms(ctx));
    double loss;
    CHECK(srhip_eval_loss(ctx, ds, P, &(srhip_loss){SRHIP_LOSS_L2, 0, 0, 0}, NULL, 0, &loss, &ok));
    STEP("tree %d: loss ok=%d loss=%.9g", t, ok, loss);
    srhip_program_destroy(P);
  }
  /* the whole batch at once */
  srhip_program* P;
  CHECK(srhip_program_create(ctx, SRHIP_F32, nodes, off, 4, &ops, &P));
  double loss[4];
  uint8_t okv[4];
  CHECK(srhip_eval_loss(ctx, ds, P, &(srhip_loss){SRHIP_LOSS_L2, 0, 0, 0}, NULL, 0, loss, okv));
  STEP("batch: loss %.9g %.9g %.9g %.9g ok %d%d%d%d", loss[0], loss[1], loss[2], loss[3], okv[0], okv[1], okv[2], okv[3]);
  srhip_program_destroy(P);
  srhip_dataset_destroy(ds);
  srhip_ctx_destroy(ctx);
  STEP("done");
  return 0;
}
