"""Derived columns: heavy unary operators applied to feature leaves are computed
once per workgroup into LDS and shared by every tree of the population.  The results must be
bit-identical to the plain program (the same operator bodies evaluate the same rows) and the
did_succeed mask must match the oracle, including columns that overflow or turn NaN."""
import os

import numpy as np
import pytest

from test_gpu_parity import F32_REL, F64_REL, _population, _rel

pytestmark = pytest.mark.gpu


def _programs(sr, ctx, nodes, offs, opts, dtype):
    """(derived program, plain program) of the same population."""
    fast = sr.Program(ctx, nodes, offs, opts, dtype)
    os.environ["SRHIP_NO_DERIVE"] = "1"
    try:
        plain = sr.Program(ctx, nodes, offs, opts, dtype)
    finally:
        del os.environ["SRHIP_NO_DERIVE"]
    assert fast.derived_columns(), "population should use derived columns"
    assert plain.derived_columns() == []
    return fast, plain


@pytest.mark.parametrize("dtype,n", [(np.float32, 1_000_000), (np.float32, 5003), (np.float64, 70_001)])
def test_derived_bit_identical_to_plain(ctx, dtype, n):
    import srhip as sr

    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("cos", "exp", "sin", "log"))
    _, nodes, offs = _population(sr, opts, 256, 5, dtype, seed=21)
    rng = np.random.default_rng(22)
    X = rng.standard_normal((5, n)).astype(dtype)
    y = (np.cos(X[1]) * X[0]).astype(dtype)
    fast, plain = _programs(sr, ctx, nodes, offs, opts, dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    a, aok = fast.eval_loss(ds, sr.L2DistLoss())
    b, bok = plain.eval_loss(ds, sr.L2DistLoss())
    assert np.array_equal(aok, bok)
    assert np.array_equal(a[aok], b[bok])
    if n <= 70_001:
        pa, pok = fast.eval_predict(ds)
        pb, _ = plain.eval_predict(ds)
        assert np.array_equal(pok, aok)
        assert np.array_equal(pa[pok].view(np.uint8), pb[pok].view(np.uint8))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_derived_nonfinite_columns_match_oracle(ctx, oracle, dtype):
    """exp of large features overflows, log / sqrt of negative ones are NaN: the trees reading
    those derived columns must fail exactly where the oracle fails."""
    import srhip as sr

    opts = sr.Options(binary_operators=("+", "-", "*", "/"), unary_operators=("exp", "log", "sqrt", "cos"))
    _, nodes, offs = _population(sr, opts, 160, 3, dtype, seed=31, max_size=12)
    rng = np.random.default_rng(32)
    n = 4099
    X = rng.standard_normal((3, n)).astype(dtype)
    X[0, 17] = 200.0 if dtype == np.float32 else 1000.0  # exp overflows in this row only
    X[2] = np.abs(X[2]) + 0.5                            # log / sqrt fine on x3 ...
    X[2, 4000] = -1.0                                     # ... except one row
    y = (X[1] * 0.5).astype(dtype)
    fast, plain = _programs(sr, ctx, nodes, offs, opts, dtype)
    ds = sr.DeviceDataset(ctx, X, y)
    dl, dok = fast.eval_loss(ds, sr.L2DistLoss())
    pl, pok = plain.eval_loss(ds, sr.L2DistLoss())
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, 0, 0.0)
    assert np.array_equal(dok, ook), np.nonzero(dok != ook)
    assert np.array_equal(dok, pok)
    assert 0 < dok.sum() < len(dok)
    tol = F32_REL if dtype == np.float32 else F64_REL
    bad = [(t, dl[t], ol[t]) for t in np.nonzero(ook)[0] if _rel(dl[t], ol[t]) > tol]
    assert not bad, bad[:5]
    assert np.array_equal(dl[dok], pl[pok])


def test_derived_with_idx_batching_and_weights(ctx, oracle):
    import srhip as sr

    opts = sr.Options(binary_operators=("+", "*", "/"), unary_operators=("cos", "exp"))
    _, nodes, offs = _population(sr, opts, 128, 4, np.float32, seed=41)
    rng = np.random.default_rng(42)
    X = rng.standard_normal((4, 9000)).astype(np.float32)
    y = rng.standard_normal(9000).astype(np.float32)
    w = np.abs(rng.standard_normal(9000)).astype(np.float32)
    idx = rng.integers(0, 9000, size=3000)
    fast, plain = _programs(sr, ctx, nodes, offs, opts, np.float32)
    ds = sr.DeviceDataset(ctx, X, y, w)
    a, aok = fast.eval_loss(ds, sr.L2DistLoss(), idx=idx)
    b, bok = plain.eval_loss(ds, sr.L2DistLoss(), idx=idx)
    assert np.array_equal(aok, bok)
    assert np.array_equal(a[aok], b[bok])
    ol, _, ook, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes,
                                           X[:, idx].copy(), y[idx].copy(), w[idx].copy(), 0, 0.0)
    assert np.array_equal(aok, ook)
    for t in np.nonzero(ook)[0]:
        assert _rel(a[t], ol[t]) < F32_REL, (t, a[t], ol[t])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_transcendentals_bitwise_at_special_values(ctx, oracle, dtype):
    """cos / sin / tan / exp on the device equal the oracle's scalar functions bit for bit at
    Inf, NaN, the fast / Payne-Hanek reduction boundary (2^28 pi/2), overflow / underflow edges and
    random arguments — through a derived column, through a plain U(x) instruction and through U of
    an operator output (x * 1), with large and small rows mixed inside a lane."""
    import srhip as sr

    special = [np.inf, -np.inf, np.nan, 4.2e8, 4.3e8, -4.3e8, 1e9, 3e38, -1e30, 88.72, 89.5, 100.0,
               -103.0, -105.0, -87.3, 1e-45, -1e-40, 0.0, -0.0, 1.5707964, 3.1415927, 1e6, 1e7 + 1]
    rng = np.random.default_rng(7)
    vals = np.concatenate([special, rng.uniform(-1e3, 1e3, 2000), rng.standard_normal(1000) * 1e7,
                           np.pi / 2 * rng.integers(-10**6, 10**6, 500)])
    X = vals.astype(dtype)[None, :]
    una = ("cos", "sin", "tan", "exp")
    opts = sr.Options(binary_operators=("*",), unary_operators=una)
    trees = [sr.Node(u, sr.Node("x1")) for u in una]                         # derived (each used twice)
    trees += [sr.Node(u, sr.Node("x1")) * 1.0 for u in una]
    trees += [sr.Node(u, sr.Node("x1") * 1.0) for u in una]                   # U of an operator output
    nodes, offs = sr.flatten(trees, opts, dtype)
    prog = sr.Program(ctx, nodes, offs, opts, dtype)
    assert len(prog.derived_columns()) == 4
    pred, _ = prog.eval_predict(sr.DeviceDataset(ctx, X))
    bits = np.uint32 if dtype == np.float32 else np.uint64
    for i, u in enumerate(una):
        code = opts.unaop_codes[opts.unary_index(u) - 1]
        ref = np.array([oracle.scalar_un(code, v, dtype) for v in X[0]], dtype=dtype)
        for t in (i, i + 4, i + 8):
            got = pred[t].astype(dtype)
            nan = np.isnan(ref)
            assert np.array_equal(np.isnan(got), nan), (u, t, X[0][np.isnan(got) != nan])
            bad = got[~nan].view(bits) != ref[~nan].view(bits)
            assert not bad.any(), (u, t, X[0][~nan][bad][:5], got[~nan][bad][:5], ref[~nan][bad][:5])
