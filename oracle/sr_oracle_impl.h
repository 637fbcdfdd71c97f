/* sr_oracle_impl.h — type-generic body of the oracle, included once per element type with
 *   T (element type), SFX (name suffix), IS_INT (0/1).
 *
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this code, and only as the checker / the CPU baseline, never as the
 * thing measured or shipped.
 *
 * A literal CPU restatement of the reference evaluator, array-at-a-time exactly as the reference
 * executes it (one fresh array per node, early return on the first failed check):
 *   DynamicExpressions.jl v0.16 eval_tree_array / _eval_tree_array / dispatch_deg1_eval /
 *   dispatch_deg2_eval / deg1_l2_ll0_lr0_eval / deg1_l1_ll0_eval / deg2_l0_r0_eval /
 *   deg2_l0_eval / deg2_r0_eval / _eval_constant_tree  (external dependency, compat "0.16",
 *   reference Project.toml:11,42; not present in the container: restated, call sites at
 *   src/InterfaceDynamicExpressions.jl:56-63), and
 *   src/LossFunctions.jl:13-33 (_loss / _weighted_loss), :45-75 (_eval_loss).
 * isfinite(sum(array)) is modelled as: every element finite AND |exact sum| below the overflow
 * threshold of T (the reference's own f32 pairwise/SIMD summation order is not reproducible and
 * is "parity unpinned" at the overflow boundary).
 */

typedef struct {
  const srhip_node* nd;
  const int32_t* binops;
  const int32_t* unaops;
  const T* X; /* [nfeat][n] */
  int64_t n;
  int64_t* done; /* nodes whose rows this evaluation produced (the early return stops it), or NULL */
} CAT(Ctx, SFX);

/* count `k` nodes evaluated over every row (cpu_baseline's work count: the reference's early
 * return skips the nodes after the first failed check) */
#define DONE(c, k) do { if ((c)->done) *(c)->done += (k); } while (0)
static int64_t CAT(subtree_size_, SFX)(const srhip_node* nd, int64_t i) {
  const srhip_node* n = &nd[i];
  if (n->degree == 0) return 1;
  if (n->degree == 1) return 1 + CAT(subtree_size_, SFX)(nd, n->l);
  return 1 + CAT(subtree_size_, SFX)(nd, n->l) + CAT(subtree_size_, SFX)(nd, n->r);
}

typedef struct {
  T* x;
  int ok;
} CAT(Res, SFX);

static T* CAT(alloc_, SFX)(int64_t n) { return (T*)malloc((size_t)(n > 0 ? n : 1) * sizeof(T)); }

static int CAT(is_const_, SFX)(const CAT(Ctx, SFX) * c, int64_t i) {
  const srhip_node* n = &c->nd[i];
  if (n->degree == 0) return n->constant;
  if (n->degree == 1) return CAT(is_const_, SFX)(c, n->l);
  return CAT(is_const_, SFX)(c, n->l) && CAT(is_const_, SFX)(c, n->r);
}

/* is_bad_array(x) = !(isempty(x) || isfinite(sum(x))) */
static int CAT(array_ok_, SFX)(const T* x, int64_t n) {
#if IS_INT
  (void)x;
  (void)n;
  return 1;
#else
  long double s = 0.0L;
  for (int64_t j = 0; j < n; ++j) {
    if (!isfinite(x[j])) return 0;
    s += (long double)x[j];
  }
  return fabsl(s) < OVF_T;
#endif
}

static int CAT(val_ok_, SFX)(T v) {
#if IS_INT
  (void)v;
  return 1;
#else
  return isfinite(v) != 0;
#endif
}

static T CAT(leaf_val_, SFX)(const srhip_node* n) { return (T)n->val; }

/* _eval_constant_tree: returns ok, value in *v (leaves are not checked) */
static int CAT(eval_const_, SFX)(const CAT(Ctx, SFX) * c, int64_t i, T* v) {
  const srhip_node* n = &c->nd[i];
  if (n->degree == 0) {
    *v = CAT(leaf_val_, SFX)(n);
    return 1;
  }
  if (n->degree == 1) {
    T a;
    if (!CAT(eval_const_, SFX)(c, n->l, &a)) return 0;
    *v = CAT(un_, SFX)(c->unaops[n->op - 1], a);
    return CAT(val_ok_, SFX)(*v);
  }
  T a, b;
  if (!CAT(eval_const_, SFX)(c, n->l, &a)) return 0;
  if (!CAT(eval_const_, SFX)(c, n->r, &b)) return 0;
  *v = CAT(bin_, SFX)(c->binops[n->op - 1], a, b);
  return CAT(val_ok_, SFX)(*v);
}

static CAT(Res, SFX) CAT(fail_, SFX)(T* x, int64_t n) {
  CAT(Res, SFX) r;
  r.x = x ? x : CAT(alloc_, SFX)(n);
  r.ok = 0;
  return r;
}

static CAT(Res, SFX) CAT(eval_, SFX)(const CAT(Ctx, SFX) * c, int64_t i);

/* deg0_eval */
static CAT(Res, SFX) CAT(deg0_, SFX)(const CAT(Ctx, SFX) * c, const srhip_node* n) {
  CAT(Res, SFX) r;
  r.x = CAT(alloc_, SFX)(c->n);
  r.ok = 1;
  DONE(c, 1);
  if (n->constant) {
    const T v = CAT(leaf_val_, SFX)(n);
    for (int64_t j = 0; j < c->n; ++j) r.x[j] = v;
  } else {
    const T* col = c->X + (int64_t)(n->feature - 1) * c->n;
    memcpy(r.x, col, (size_t)c->n * sizeof(T));
  }
  return r;
}

static T CAT(leafrow_, SFX)(const CAT(Ctx, SFX) * c, const srhip_node* n, int64_t j) {
  return n->constant ? CAT(leaf_val_, SFX)(n) : c->X[(int64_t)(n->feature - 1) * c->n + j];
}

#if IS_INT
#define INF_T ((T)0)
#define NONFINITE(x) 0
#else
#define INF_T ((T)INFINITY)
#define NONFINITE(x) (!isfinite(x))
#endif

static CAT(Res, SFX) CAT(dispatch_deg1_, SFX)(const CAT(Ctx, SFX) * c, int64_t i) {
  const srhip_node* n = &c->nd[i];
  const int op = c->unaops[n->op - 1];
  const srhip_node* l = &c->nd[n->l];
  if (l->degree == 2 && c->nd[l->l].degree == 0 && c->nd[l->r].degree == 0) {
    /* deg1_l2_ll0_lr0_eval: op(op_l(x, y)) with x, y leaves */
    const int op_l = c->binops[l->op - 1];
    const srhip_node* ll = &c->nd[l->l];
    const srhip_node* lr = &c->nd[l->r];
    if (ll->constant && !CAT(val_ok_, SFX)(CAT(leaf_val_, SFX)(ll))) return CAT(fail_, SFX)(NULL, c->n);
    if (lr->constant && !CAT(val_ok_, SFX)(CAT(leaf_val_, SFX)(lr))) return CAT(fail_, SFX)(NULL, c->n);
    CAT(Res, SFX) r;
    r.x = CAT(alloc_, SFX)(c->n);
    r.ok = 1;
    for (int64_t j = 0; j < c->n; ++j) {
      const T xl = CAT(bin_, SFX)(op_l, CAT(leafrow_, SFX)(c, ll, j), CAT(leafrow_, SFX)(c, lr, j));
      r.x[j] = NONFINITE(xl) ? INF_T : CAT(un_, SFX)(op, xl);
    }
    DONE(c, 4);
    return r;
  }
  if (l->degree == 1 && c->nd[l->l].degree == 0) {
    /* deg1_l1_ll0_eval: op(op_l(x)) with x a leaf */
    const int op_l = c->unaops[l->op - 1];
    const srhip_node* ll = &c->nd[l->l];
    if (ll->constant && !CAT(val_ok_, SFX)(CAT(leaf_val_, SFX)(ll))) return CAT(fail_, SFX)(NULL, c->n);
    CAT(Res, SFX) r;
    r.x = CAT(alloc_, SFX)(c->n);
    r.ok = 1;
    for (int64_t j = 0; j < c->n; ++j) {
      const T xl = CAT(un_, SFX)(op_l, CAT(leafrow_, SFX)(c, ll, j));
      r.x[j] = NONFINITE(xl) ? INF_T : CAT(un_, SFX)(op, xl);
    }
    DONE(c, 3);
    return r;
  }
  /* op(x) for any x */
  CAT(Res, SFX) r = CAT(eval_, SFX)(c, n->l);
  if (!r.ok) return r;
  if (!CAT(array_ok_, SFX)(r.x, c->n)) {
    r.ok = 0;
    return r;
  }
  for (int64_t j = 0; j < c->n; ++j) r.x[j] = CAT(un_, SFX)(op, r.x[j]);
  DONE(c, 1);
  return r;
}

static CAT(Res, SFX) CAT(dispatch_deg2_, SFX)(const CAT(Ctx, SFX) * c, int64_t i) {
  const srhip_node* n = &c->nd[i];
  const int op = c->binops[n->op - 1];
  const srhip_node* l = &c->nd[n->l];
  const srhip_node* rr = &c->nd[n->r];
  if (l->degree == 0 && rr->degree == 0) {
    /* deg2_l0_r0_eval */
    if (l->constant && !CAT(val_ok_, SFX)(CAT(leaf_val_, SFX)(l))) return CAT(fail_, SFX)(NULL, c->n);
    if (rr->constant && !CAT(val_ok_, SFX)(CAT(leaf_val_, SFX)(rr))) return CAT(fail_, SFX)(NULL, c->n);
    CAT(Res, SFX) r;
    r.x = CAT(alloc_, SFX)(c->n);
    r.ok = 1;
    for (int64_t j = 0; j < c->n; ++j)
      r.x[j] = CAT(bin_, SFX)(op, CAT(leafrow_, SFX)(c, l, j), CAT(leafrow_, SFX)(c, rr, j));
    DONE(c, 3);
    return r;
  }
  if (rr->degree == 0) {
    /* deg2_r0_eval: op(x, y) with y a leaf */
    CAT(Res, SFX) L = CAT(eval_, SFX)(c, n->l);
    if (!L.ok) return L;
    if (!CAT(array_ok_, SFX)(L.x, c->n)) {
      L.ok = 0;
      return L;
    }
    if (rr->constant && !CAT(val_ok_, SFX)(CAT(leaf_val_, SFX)(rr))) {
      L.ok = 0;
      return L;
    }
    for (int64_t j = 0; j < c->n; ++j) L.x[j] = CAT(bin_, SFX)(op, L.x[j], CAT(leafrow_, SFX)(c, rr, j));
    DONE(c, 2);
    return L;
  }
  if (l->degree == 0) {
    /* deg2_l0_eval: op(x, y) with x a leaf */
    CAT(Res, SFX) R = CAT(eval_, SFX)(c, n->r);
    if (!R.ok) return R;
    if (!CAT(array_ok_, SFX)(R.x, c->n)) {
      R.ok = 0;
      return R;
    }
    if (l->constant && !CAT(val_ok_, SFX)(CAT(leaf_val_, SFX)(l))) {
      R.ok = 0;
      return R;
    }
    for (int64_t j = 0; j < c->n; ++j) R.x[j] = CAT(bin_, SFX)(op, CAT(leafrow_, SFX)(c, l, j), R.x[j]);
    DONE(c, 2);
    return R;
  }
  CAT(Res, SFX) L = CAT(eval_, SFX)(c, n->l);
  if (!L.ok) return L;
  if (!CAT(array_ok_, SFX)(L.x, c->n)) {
    L.ok = 0;
    return L;
  }
  CAT(Res, SFX) R = CAT(eval_, SFX)(c, n->r);
  if (!R.ok) {
    free(L.x);
    return R;
  }
  if (!CAT(array_ok_, SFX)(R.x, c->n)) {
    free(L.x);
    R.ok = 0;
    return R;
  }
  for (int64_t j = 0; j < c->n; ++j) L.x[j] = CAT(bin_, SFX)(op, L.x[j], R.x[j]);
  free(R.x);
  DONE(c, 1);
  return L;
}

/* _eval_tree_array */
static CAT(Res, SFX) CAT(eval_, SFX)(const CAT(Ctx, SFX) * c, int64_t i) {
  const srhip_node* n = &c->nd[i];
  if (n->degree == 0) return CAT(deg0_, SFX)(c, n);
  if (CAT(is_const_, SFX)(c, i)) {
    T v;
    if (!CAT(eval_const_, SFX)(c, i, &v)) return CAT(fail_, SFX)(NULL, c->n);
    CAT(Res, SFX) r;
    r.x = CAT(alloc_, SFX)(c->n);
    r.ok = 1;
    for (int64_t j = 0; j < c->n; ++j) r.x[j] = v;
    DONE(c, CAT(subtree_size_, SFX)(c->nd, i));
    return r;
  }
  if (n->degree == 1) return CAT(dispatch_deg1_, SFX)(c, i);
  return CAT(dispatch_deg2_, SFX)(c, i);
}

/* eval_tree_array(tree, X, operators) -> (out, ok); X is [nfeat][n] (SoA). out may be NULL.
 * *done (nullable) += the nodes evaluated over all rows before the result or the early return. */
static int CAT(eval_tree_work_, SFX)(const srhip_node* nodes, const int32_t* binops, const int32_t* unaops,
                                     const T* X, int64_t n, T* out, int64_t* done) {
  CAT(Ctx, SFX) c;
  c.nd = nodes;
  c.binops = binops;
  c.unaops = unaops;
  c.X = X;
  c.n = n;
  c.done = done;
  CAT(Res, SFX) r = CAT(eval_, SFX)(&c, 0);
  int ok = r.ok && CAT(array_ok_, SFX)(r.x, n);
  if (out) memcpy(out, r.x, (size_t)n * sizeof(T));
  free(r.x);
  return ok;
}
int CAT(oracle_eval_tree_, SFX)(const srhip_node* nodes, const int32_t* binops, const int32_t* unaops, const T* X,
                                int64_t n, T* out) {
  return CAT(eval_tree_work_, SFX)(nodes, binops, unaops, X, n, out, NULL);
}

/* _eval_loss(tree, dataset, options; regularization=false):
 *   loss_exact = (sum_i w_i l_i) / (sum_i w_i)   in long double (the parity target)
 *   loss_ref   = the reference's own order: sequential fold in T of l_i (mean), or
 *                sum(w .* l) / sum(w) with both sums folded sequentially in T
 * returns ok (did_succeed); losses are +Inf when !ok. */
static int CAT(eval_loss_work_, SFX)(const srhip_node* nodes, const int32_t* binops, const int32_t* unaops,
                                     const T* X, const T* y, const T* w, int64_t n, int loss_kind, double p0,
                                     double* loss_exact, double* loss_ref, int64_t* done) {
  T* pred = CAT(alloc_, SFX)(n);
  int ok = CAT(eval_tree_work_, SFX)(nodes, binops, unaops, X, n, pred, done);
  if (!ok) {
    free(pred);
    if (loss_exact) *loss_exact = INFINITY;
    if (loss_ref) *loss_ref = INFINITY;
    return 0;
  }
#if IS_INT
  long long s = 0;
  for (int64_t j = 0; j < n; ++j) {
    const int32_t d = (int32_t)((uint32_t)pred[j] - (uint32_t)y[j]);
    int32_t l = loss_kind == SRHIP_LOSS_L1 ? (d < 0 ? (int32_t)(0u - (uint32_t)d) : d) : (int32_t)((uint32_t)d * (uint32_t)d);
    s += l;
  }
  (void)w;
  (void)p0;
  if (loss_exact) *loss_exact = (double)s / (double)n;
  if (loss_ref) *loss_ref = (double)s / (double)n;
#else
  long double se = 0.0L, swe = 0.0L;
  T sr = 0, swr = 0;
  for (int64_t j = 0; j < n; ++j) {
    const T l = CAT(loss_, SFX)(loss_kind, pred[j], y[j], (T)p0);
    if (w) {
      const T wl = w[j] * l;
      se += (long double)wl;
      swe += (long double)w[j];
      sr = j == 0 ? wl : sr + wl;
      swr = j == 0 ? w[j] : swr + w[j];
    } else {
      se += (long double)l;
      sr = j == 0 ? l : sr + l;
    }
  }
  if (loss_exact) *loss_exact = (double)(w ? se / swe : se / (long double)n);
  if (loss_ref) *loss_ref = (double)(w ? sr / swr : sr / (T)n);
#endif
  free(pred);
  return 1;
}
int CAT(oracle_eval_loss_, SFX)(const srhip_node* nodes, const int32_t* binops, const int32_t* unaops, const T* X,
                                const T* y, const T* w, int64_t n, int loss_kind, double p0, double* loss_exact,
                                double* loss_ref) {
  return CAT(eval_loss_work_, SFX)(nodes, binops, unaops, X, y, w, n, loss_kind, p0, loss_exact, loss_ref, NULL);
}

/* Batched: every tree of a population (threads across trees, as the reference's
 * :multithreading runs one task per population).  Returns the number of threads used. */
int CAT(oracle_eval_loss_batch_work_, SFX)(const srhip_node* nodes, const int64_t* offsets, int32_t ntrees,
                                           const int32_t* binops, const int32_t* unaops, const T* X, const T* y,
                                           const T* w, int64_t n, int loss_kind, double p0, int nthreads,
                                           double* loss_exact, double* loss_ref, uint8_t* ok, int64_t* node_rows) {
  int used = 1;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
  {
#pragma omp single
    used = omp_get_num_threads();
#pragma omp for schedule(dynamic, 1)
    for (int32_t t = 0; t < ntrees; ++t) {
      double le, lr;
      int64_t done = 0;
      ok[t] = (uint8_t)CAT(eval_loss_work_, SFX)(nodes + offsets[t], binops, unaops, X, y, w, n, loss_kind, p0, &le, &lr, &done);
      if (node_rows) node_rows[t] = done * n;
      loss_exact[t] = le;
      if (loss_ref) loss_ref[t] = lr;
    }
  }
#else
  (void)nthreads;
  for (int32_t t = 0; t < ntrees; ++t) {
    double le, lr;
    int64_t done = 0;
    ok[t] = (uint8_t)CAT(eval_loss_work_, SFX)(nodes + offsets[t], binops, unaops, X, y, w, n, loss_kind, p0, &le, &lr, &done);
    if (node_rows) node_rows[t] = done * n;
    loss_exact[t] = le;
    if (loss_ref) loss_ref[t] = lr;
  }
#endif
  return used;
}

int CAT(oracle_eval_loss_batch_, SFX)(const srhip_node* nodes, const int64_t* offsets, int32_t ntrees,
                                      const int32_t* binops, const int32_t* unaops, const T* X, const T* y,
                                      const T* w, int64_t n, int loss_kind, double p0, int nthreads,
                                      double* loss_exact, double* loss_ref, uint8_t* ok) {
  return CAT(oracle_eval_loss_batch_work_, SFX)(nodes, offsets, ntrees, binops, unaops, X, y, w, n, loss_kind, p0,
                                                nthreads, loss_exact, loss_ref, ok, NULL);
}

#undef INF_T
#undef NONFINITE
#undef DONE

/* ---- row-shard partials (test infrastructure for the multi-GPU protocol, include/srhip.h) ----
 * Row-wise restatement of what one shard contributes: per tree {sum (w*)loss, sum w (or rows)},
 * per feature {column sum (Float64: x * 2^-64), non-finite count}, rows; chk[t] = max |v| (Float32,
 * NaN-propagating) or sum |v| 2^-512 (Float64) over the outputs of every non-constant operator
 * node (constant subtrees are scalars in the reference and on the device). */
static T CAT(rowval_, SFX)(const CAT(Ctx, SFX) * c, int64_t i, int64_t j, double* chk, int* chk_nan) {
  const srhip_node* n = &c->nd[i];
  if (n->degree == 0) return CAT(leafrow_, SFX)(c, n, j);
  if (CAT(is_const_, SFX)(c, i)) {
    T v = 0;
    CAT(eval_const_, SFX)(c, i, &v);
    return v;
  }
  T v;
  if (n->degree == 1) {
    v = CAT(un_, SFX)(c->unaops[n->op - 1], CAT(rowval_, SFX)(c, n->l, j, chk, chk_nan));
  } else {
    const T a = CAT(rowval_, SFX)(c, n->l, j, chk, chk_nan);
    const T b = CAT(rowval_, SFX)(c, n->r, j, chk, chk_nan);
    v = CAT(bin_, SFX)(c->binops[n->op - 1], a, b);
  }
#if !IS_INT
  if (v != v) *chk_nan = 1;
  const double av = fabs((double)v);
  if (sizeof(T) == 8) *chk += av * 0x1p-512;
  else if (av > *chk) *chk = av;
#endif
  return v;
}

void CAT(oracle_partials_, SFX)(const srhip_node* nodes, const int64_t* offsets, int32_t ntrees, const int32_t* binops,
                                const int32_t* unaops, const T* X, int64_t nfeat, const T* y, const T* w, int64_t n,
                                int loss_kind, double p0, double* sums, double* chk) {
  for (int32_t t = 0; t < ntrees; ++t) {
    CAT(Ctx, SFX) c;
    c.nd = nodes + offsets[t];
    c.binops = binops;
    c.unaops = unaops;
    c.X = X;
    c.n = n;
    c.done = NULL;
    long double ls = 0.0L, ws = 0.0L;
    double ck = 0.0;
    int ck_nan = 0;
    for (int64_t j = 0; j < n; ++j) {
      const T pv = CAT(rowval_, SFX)(&c, 0, j, &ck, &ck_nan);
#if IS_INT
      const int32_t d = (int32_t)((uint32_t)pv - (uint32_t)y[j]);
      ls += loss_kind == SRHIP_LOSS_L1 ? (d < 0 ? -(long double)d : (long double)d) : (long double)(int32_t)((uint32_t)d * (uint32_t)d);
      ws += 1.0L;
#else
      const T l = CAT(loss_, SFX)(loss_kind, pv, y[j], (T)p0);
      if (w) {
        ls += (long double)(w[j] * l);
        ws += (long double)w[j];
      } else {
        ls += (long double)l;
        ws += 1.0L;
      }
#endif
    }
    sums[2 * t] = (double)ls;
    sums[2 * t + 1] = (double)ws;
    chk[t] = ck_nan ? (double)NAN : ck;
  }
  for (int64_t f = 0; f < nfeat; ++f) {
    long double s = 0.0L;
    double bad = 0;
    for (int64_t j = 0; j < n; ++j) {
      const T v = X[f * n + j];
#if IS_INT
      s += (long double)v;
#else
      if (!isfinite(v)) bad += 1;
      else s += sizeof(T) == 8 ? (long double)v * 0x1p-64L : (long double)v;
#endif
    }
    sums[2 * (int64_t)ntrees + 2 * f] = (double)s;
    sums[2 * (int64_t)ntrees + 2 * f + 1] = bad;
  }
  sums[2 * (int64_t)ntrees + 2 * nfeat] = (double)n;
}
