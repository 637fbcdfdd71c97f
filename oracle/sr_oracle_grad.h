/* sr_oracle_grad.h — ORACLE, TEST INFRASTRUCTURE ONLY (included by sr_oracle.c; see its header).
 *
 * The exact gradient of _eval_loss(regularization=false) (src/LossFunctions.jl:45-75) with respect
 * to a tree's constants in get_constants order (depth-first, left to right: src/ConstantOptimization.jl
 * :46-50 via DynamicExpressions get_constants), by forward-mode dual numbers, row by row: every
 * node's value is the value oracle's (un_f64 / bin_f64: the same operator semantics and libm), its
 * tangent the chain rule with the partial derivatives below, and the loss gradient
 * (1/sum w) sum_rows w_i l'(pred_i - y_i) d pred_i / d c, summed in long double.
 * Used by oracle/optim.py's exact-gradient mode: the reference differentiates by finite
 * differences (Optim with only f, FiniteDiff central steps); libsrhip differentiates exactly (dual
 * numbers), so the optimiser's state machine is checked against a restatement that differentiates
 * exactly too, and the finite-difference restatement stays the reference-deviation check.
 * Float64 trees; + - * / pow, and the unary operators with a derivative below (others: NaN).
 */
#define GRAD_MAXC 64

typedef struct {
  const srhip_node* nd;
  const int32_t* binops;
  const int32_t* unaops;
  const double* X; /* [nfeat][n] */
  int64_t n, row;
  int nc;
  const int32_t* cidx; /* constant index of each node, -1 otherwise */
} GradCtx;

/* value of node i at ctx->row; its tangent (nc components) in t */
static double grad_node(const GradCtx* c, int64_t i, double* t) {
  const srhip_node* n = &c->nd[i];
  if (n->degree == 0) {
    for (int k = 0; k < c->nc; ++k) t[k] = 0.0;
    if (n->constant) {
      t[c->cidx[i]] = 1.0;
      return n->val;
    }
    return c->X[(int64_t)(n->feature - 1) * c->n + c->row];
  }
  if (n->degree == 1) {
    const double x = grad_node(c, n->l, t);
    const int op = c->unaops[n->op - 1];
    const double f = un_f64(op, x);
    double df;
    switch (op) {
      case SRHIP_OP_NEG: df = -1.0; break;
      case SRHIP_OP_SQUARE: df = 2.0 * x; break;
      case SRHIP_OP_CUBE: df = 3.0 * x * x; break;
      case SRHIP_OP_ABS: df = x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : 0.0); break;
      case SRHIP_OP_COS: df = -srm_sin(x); break;
      case SRHIP_OP_SIN: df = srm_cos(x); break;
      case SRHIP_OP_TAN: df = 1.0 + f * f; break;
      case SRHIP_OP_EXP: df = f; break;
      case SRHIP_OP_LOG: df = 1.0 / x; break;
      case SRHIP_OP_SQRT: df = 0.5 / f; break;
      case SRHIP_OP_TANH: df = 1.0 - f * f; break;
      default: df = NAN; break;
    }
    for (int k = 0; k < c->nc; ++k) t[k] = df * t[k];
    return f;
  }
  double tr[GRAD_MAXC];
  const double a = grad_node(c, n->l, t);
  const double b = grad_node(c, n->r, tr);
  const int op = c->binops[n->op - 1];
  const double f = bin_f64(op, a, b);
  double fa, fb;
  switch (op) {
    case SRHIP_OP_ADD: fa = 1.0; fb = 1.0; break;
    case SRHIP_OP_SUB: fa = 1.0; fb = -1.0; break;
    case SRHIP_OP_MUL: fa = b; fb = a; break;
    case SRHIP_OP_DIV: { const double ib = 1.0 / b; fa = ib; fb = -f * ib; break; }
    case SRHIP_OP_POW: fa = b * bin_f64(SRHIP_OP_POW, a, b - 1.0); fb = a > 0.0 ? f * srm_log(a) : 0.0; break;
    default: fa = NAN; fb = NAN; break;
  }
  for (int k = 0; k < c->nc; ++k) t[k] = fa * t[k] + fb * tr[k];
  return f;
}

static void grad_const_index(const srhip_node* nd, int64_t i, int32_t* cidx, int* next) {
  const srhip_node* n = &nd[i];
  if (n->degree == 0) {
    if (n->constant) cidx[i] = (*next)++;
    return;
  }
  grad_const_index(nd, n->l, cidx, next);
  if (n->degree == 2) grad_const_index(nd, n->r, cidx, next);
}

/* One Float64 tree (nodes[0..nn)), L2 / L1 loss (kind), optional weights: out_grad[nconst] =
 * d loss / d c.  Returns the number of constants, or -1 if more than GRAD_MAXC. */
int oracle_loss_grad_f64(const srhip_node* nodes, int64_t nn, const int32_t* binops, const int32_t* unaops,
                         const double* X, const double* y, const double* w, int64_t n, int kind, double* out_grad) {
  int32_t* cidx = (int32_t*)malloc((size_t)(nn > 0 ? nn : 1) * sizeof(int32_t));
  for (int64_t i = 0; i < nn; ++i) cidx[i] = -1;
  int nc = 0;
  grad_const_index(nodes, 0, cidx, &nc);
  if (nc > GRAD_MAXC) {
    free(cidx);
    return -1;
  }
  GradCtx c = {nodes, binops, unaops, X, n, 0, nc, cidx};
  long double acc[GRAD_MAXC], wsum = 0.0L;
  double t[GRAD_MAXC];
  for (int k = 0; k < nc; ++k) acc[k] = 0.0L;
  for (int64_t r = 0; r < n; ++r) {
    c.row = r;
    const double pred = grad_node(&c, 0, t);
    const double d = pred - y[r];
    double dl = kind == SRHIP_LOSS_L1 ? (d > 0.0 ? 1.0 : (d < 0.0 ? -1.0 : 0.0)) : 2.0 * d;
    const double wr = w ? w[r] : 1.0;
    if (w) dl = wr * dl;
    for (int k = 0; k < nc; ++k) acc[k] += (long double)(dl * t[k]);
    wsum += (long double)wr;
  }
  for (int k = 0; k < nc; ++k) out_grad[k] = (double)(acc[k] / wsum);
  free(cidx);
  return nc;
}

/* ---- the device's row-sum order (libsrhip's dual-number kernel, csrc/srhip_grad.hip) -----------
 * Exact sums make the optimiser's trajectory chaotic wherever a line search compares phi values at
 * the rounding noise (tiny steps): to compare the device optimiser's state machine bit for bit, the
 * exact-gradient restatement can sum its per-row values in the order the device kernel does: row
 * blocks of rb rows; in a block each of 64 lanes adds rows (block + 64 j + lane), j ascending, from
 * 0.0; the 64 lane sums fold by the xor butterfly (offsets 32, 16, ..., 1); the block sums fold per
 * lane l over blocks l, l + 64, ... ascending, then the same butterfly; the result is lane 0's. */
static void dev_butterfly(double* s) {
  for (int o = 32; o > 0; o >>= 1) {
    double t[64];
    for (int l = 0; l < 64; ++l) t[l] = s[l] + s[l ^ o];
    for (int l = 0; l < 64; ++l) s[l] = t[l];
  }
}
static double dev_order_sum(const double* v, int64_t n, int64_t stride, int rb) {
  const int64_t nrb = (n + rb - 1) / rb;
  double red[64];
  for (int l = 0; l < 64; ++l) red[l] = 0.0;
  for (int64_t b = 0; b < nrb; ++b) {
    double s[64];
    for (int l = 0; l < 64; ++l) s[l] = 0.0;
    for (int64_t j = 0; j < rb; j += 64)
      for (int l = 0; l < 64; ++l) {
        const int64_t r = b * rb + j + l;
        if (r < n) s[l] += v[r * stride];
      }
    dev_butterfly(s);
    red[b % 64] += s[0];
  }
  dev_butterfly(red);
  return red[0];
}

/* Loss sum and gradient (out[0] = sum of row losses / sum w, out[1 + k] = d loss / d c_k) of one
 * Float64 tree with the device kernel's row-sum order (rb rows per block: libsrhip's grad_plan, 256).
 * Returns the number of constants, or -1. */
int oracle_loss_grad_devorder_f64(const srhip_node* nodes, int64_t nn, const int32_t* binops,
                                  const int32_t* unaops, const double* X, const double* y, const double* w,
                                  int64_t n, int kind, int rb, double* out) {
  int32_t* cidx = (int32_t*)malloc((size_t)(nn > 0 ? nn : 1) * sizeof(int32_t));
  for (int64_t i = 0; i < nn; ++i) cidx[i] = -1;
  int nc = 0;
  grad_const_index(nodes, 0, cidx, &nc);
  if (nc > GRAD_MAXC) {
    free(cidx);
    return -1;
  }
  const int64_t stride = nc + 1;
  double* rows = (double*)malloc((size_t)(n > 0 ? n : 1) * stride * sizeof(double));
  GradCtx c = {nodes, binops, unaops, X, n, 0, nc, cidx};
  double t[GRAD_MAXC], wsum = 0.0;
  for (int64_t r = 0; r < n; ++r) {
    c.row = r;
    const double pred = grad_node(&c, 0, t);
    const double d = pred - y[r];
    double l = kind == SRHIP_LOSS_L1 ? fabs(d) : d * d;
    double dl = kind == SRHIP_LOSS_L1 ? (d > 0.0 ? 1.0 : (d < 0.0 ? -1.0 : 0.0)) : 2.0 * d;
    if (w) {
      l = w[r] * l;
      dl = w[r] * dl;
    }
    rows[r * stride] = l;
    for (int k = 0; k < nc; ++k) rows[r * stride + 1 + k] = dl * t[k];
  }
  if (w) {
    for (int64_t r = 0; r < n; ++r) wsum += w[r];  /* the host's sum of the weights */
  } else {
    wsum = (double)n;
  }
  for (int k = 0; k <= nc; ++k) out[k] = dev_order_sum(rows + k, n, stride, rb) / wsum;
  free(rows);
  free(cidx);
  return nc;
}

/* ---- Float32 trees: the dual-number kernel's Float32 arithmetic, device row order ---------------
 * libsrhip's constant optimiser treats a Float32 program as the reference's Float32 tree: every
 * objective call evaluates the tree with its constants rounded to Float32, the values and tangents in
 * Float32 (csrc/srhip_grad.hip dual_un_heavy / dual_spec / combine: the same products and sums, no
 * contraction), the per-row loss l = d * d and dl = 2 d in Float32, and the row sums (double)l,
 * (double)(dl * t_k) in the device's order (dev_order_sum above). */
static float grad_node_f32(const GradCtx* c, const float* X32, int64_t i, float* t) {
  const srhip_node* n = &c->nd[i];
  if (n->degree == 0) {
    for (int k = 0; k < c->nc; ++k) t[k] = 0.0f;
    if (n->constant) {
      t[c->cidx[i]] = 1.0f;
      return (float)n->val;
    }
    return X32[(int64_t)(n->feature - 1) * c->n + c->row];
  }
  if (n->degree == 1) {
    const float x = grad_node_f32(c, X32, n->l, t);
    const int op = c->unaops[n->op - 1];
    const float f = un_f32(op, x);
    float df;
    switch (op) {
      case SRHIP_OP_NEG: df = -1.0f; break;
      case SRHIP_OP_SQUARE: df = 2.0f * x; break;
      case SRHIP_OP_CUBE: df = 3.0f * x * x; break;
      case SRHIP_OP_ABS: df = x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); break;
      case SRHIP_OP_COS: df = -srm_sinf(x); break;
      case SRHIP_OP_SIN: df = srm_cosf(x); break;
      case SRHIP_OP_TAN: df = 1.0f + f * f; break;
      case SRHIP_OP_EXP: df = f; break;
      case SRHIP_OP_LOG: df = 1.0f / x; break;
      case SRHIP_OP_SQRT: df = 0.5f / f; break;
      case SRHIP_OP_TANH: df = 1.0f - f * f; break;
      default: df = NAN; break;
    }
    for (int k = 0; k < c->nc; ++k) t[k] = df * t[k];
    return f;
  }
  float tr[GRAD_MAXC];
  const float a = grad_node_f32(c, X32, n->l, t);
  const float b = grad_node_f32(c, X32, n->r, tr);
  const int op = c->binops[n->op - 1];
  const float f = bin_f32(op, a, b);
  float fa, fb;
  switch (op) {
    case SRHIP_OP_ADD: fa = 1.0f; fb = 1.0f; break;
    case SRHIP_OP_SUB: fa = 1.0f; fb = -1.0f; break;
    case SRHIP_OP_MUL: fa = b; fb = a; break;
    case SRHIP_OP_DIV: { const float ib = 1.0f / b; fa = ib; fb = -f * ib; break; }
    default: fa = NAN; fb = NAN; break;
  }
  for (int k = 0; k < c->nc; ++k) t[k] = fa * t[k] + fb * tr[k];
  return f;
}

/* oracle_loss_grad_devorder_f64's Float32 counterpart: nodes' constants are rounded to Float32 as the
 * device's program holds them; X, y, w are Float32; out as there (f64). */
int oracle_loss_grad_devorder_f32(const srhip_node* nodes, int64_t nn, const int32_t* binops,
                                  const int32_t* unaops, const float* X, const float* y, const float* w,
                                  int64_t n, int kind, int rb, double* out) {
  int32_t* cidx = (int32_t*)malloc((size_t)(nn > 0 ? nn : 1) * sizeof(int32_t));
  for (int64_t i = 0; i < nn; ++i) cidx[i] = -1;
  int nc = 0;
  grad_const_index(nodes, 0, cidx, &nc);
  if (nc > GRAD_MAXC) {
    free(cidx);
    return -1;
  }
  const int64_t stride = nc + 1;
  double* rows = (double*)malloc((size_t)(n > 0 ? n : 1) * stride * sizeof(double));
  GradCtx c = {nodes, binops, unaops, NULL, n, 0, nc, cidx};
  float t[GRAD_MAXC];
  double wsum = 0.0;
  for (int64_t r = 0; r < n; ++r) {
    c.row = r;
    const float pred = grad_node_f32(&c, X, 0, t);
    const float d = pred - y[r];
    float l = kind == SRHIP_LOSS_L1 ? fabsf(d) : d * d;
    float dl = kind == SRHIP_LOSS_L1 ? (d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f)) : 2.0f * d;
    if (w) {
      l = w[r] * l;
      dl = w[r] * dl;
    }
    rows[r * stride] = (double)l;
    for (int k = 0; k < nc; ++k) rows[r * stride + 1 + k] = (double)(dl * t[k]);
  }
  if (w) {
    for (int64_t r = 0; r < n; ++r) wsum += (double)w[r];
  } else {
    wsum = (double)n;
  }
  for (int k = 0; k <= nc; ++k) out[k] = dev_order_sum(rows + k, n, stride, rb) / wsum;
  free(rows);
  free(cidx);
  return nc;
}
