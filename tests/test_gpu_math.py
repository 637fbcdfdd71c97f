"""The DEVICE's transcendentals, pinned independently of the header they share with the oracle
(include/srhip_math.h is compiled by hipcc for the kernels and by gcc for the oracle, so the
oracle-vs-device parity tests cannot see an accuracy defect of the shared code, or a defect only the
device build has).  Single-operator trees exp / log / sin / cos / tan run through
srhip_eval_predict (the interpreter and, for U(x1), the derived-column path) on >= 1e6 inputs per
(operator, type) -- ordinary, huge and special arguments -- and are compared with glibc through
numpy (Float64: <= 1 ULP, tan <= 2) and with mpmath's correctly rounded value (Float32: <= 1 ULP,
< 1 % of inputs differing; exp, Julia's 1-ULP Float32 algorithm: < 15 %), the bounds
tests/test_math_accuracy.py asserts for the CPU build.  test_device_float32_exp_bits_equal_oracle
compares the device's packed exp with the oracle's scalar one bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
mpmath = pytest.importorskip("mpmath")

NAMES = ("exp", "log", "sin", "cos", "tan")
RNG = np.random.default_rng(2026)


def _ulps64(a, b):
    ai, bi = a.view(np.int64), b.view(np.int64)
    ai = np.where(ai < 0, np.int64(-(2**63)) - ai, ai)
    bi = np.where(bi < 0, np.int64(-(2**63)) - bi, bi)
    return np.abs(ai - bi)


def _ulps32(a, b):
    ai, bi = a.view(np.int32).astype(np.int64), b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(1 << 31) - ai, ai)
    bi = np.where(bi < 0, -(1 << 31) - bi, bi)
    return np.abs(ai - bi)


def _inputs64(name, n=1_200_000):
    if name == "exp":
        parts = [RNG.uniform(-745, 709.7, n // 2), RNG.uniform(-1, 1, n // 2)]
    elif name == "log":
        parts = [np.exp(RNG.uniform(-700, 700, n // 2)), RNG.uniform(0.9, 1.1, n // 2),
                 np.array([5e-324, 1e-310, 2.2250738585072014e-308, 1.0, 2.0, 1.7976931348623157e308])]
    else:
        parts = [RNG.uniform(-10, 10, n // 2), RNG.uniform(-2e6, 2e6, n // 4),
                 10 ** RNG.uniform(6, 300, n // 4) * RNG.choice([-1, 1], n // 4)]
    return np.concatenate(parts)


def _inputs32(name, n=1_200_000):
    if name == "exp":
        x = RNG.uniform(-104, 89, n)
    elif name == "log":
        x = np.exp(RNG.uniform(-100, 88, n))
    elif name == "tan":
        x = np.concatenate([RNG.uniform(-8, 8, n // 2), RNG.uniform(-1e5, 1e5, n // 4), 10 ** RNG.uniform(5, 38, n // 4)])
    else:
        x = np.concatenate([RNG.uniform(-8, 8, n // 2), RNG.uniform(-1e5, 1e5, n // 4), 10 ** RNG.uniform(5, 38, n // 4)])
    return x.astype(np.float32)


def _device(ctx, name, x):
    import srhip

    opts = srhip.Options(binary_operators=("+",), unary_operators=NAMES)
    tree = srhip.Node(name, srhip.Node("x1"))
    nodes, offs = srhip.flatten([tree], opts, x.dtype)
    prog = srhip.Program(ctx, nodes, offs, opts, x.dtype)
    pred, _ = prog.eval_predict(srhip.DeviceDataset(ctx, x[None, :]))
    return pred[0]


@pytest.mark.parametrize("name", NAMES)
def test_device_float64_within_ulp_of_glibc(ctx, name):
    x = _inputs64(name)
    got = _device(ctx, name, x)
    ref = getattr(np, name)(x)
    u = _ulps64(got, ref)
    assert u.max() <= (2 if name == "tan" else 1), (name, x[np.argmax(u)], got[np.argmax(u)], ref[np.argmax(u)])


@pytest.mark.parametrize("name", NAMES)
def test_device_float32_vs_correctly_rounded(ctx, name):
    x = _inputs32(name)
    got = _device(ctx, name, x)
    # every input against glibc in Float64 rounded once (itself within 1/2 ULP + 2^-52 relative);
    # exp is Julia's 1-ULP Float32 algorithm (~8 % of these arguments round the other way)
    differ = 0.15 if name == "exp" else 0.01
    ref = getattr(np, name)(x.astype(np.float64)).astype(np.float32)
    u = _ulps32(got, ref)
    assert u.max() <= 1, (name, x[np.argmax(u)])
    assert np.mean(u > 0) < differ, np.mean(u > 0)
    # a sample against the correctly rounded value (mpmath, 200 bits)
    mpmath.mp.prec = 200
    idx = RNG.choice(len(x), 4000, replace=False)
    fn = getattr(mpmath, name)
    cr = np.array([float(fn(mpmath.mpf(float(v)))) for v in x[idx]]).astype(np.float32)
    u = _ulps32(got[idx], cr)
    assert u.max() <= 1, (name, x[idx][np.argmax(u)])
    assert np.mean(u > 0) < differ


def test_device_special_values(ctx):
    inf, nan = np.inf, np.nan
    for dt in (np.float32, np.float64):
        e = _device(ctx, "exp", np.array([inf, -inf, nan, 0.0, -0.0, 1e4, -1e4], dtype=dt))
        assert e[0] == inf and e[1] == 0 and np.isnan(e[2]) and e[3] == 1 and e[4] == 1 and e[5] == inf and e[6] == 0
        lg = _device(ctx, "log", np.array([0.0, -1.0, inf, nan, 1.0], dtype=dt))
        assert np.all(np.isnan(lg[:2])) and lg[2] == inf and np.isnan(lg[3]) and lg[4] == 0  # safe_log: x <= 0 -> NaN
        for name in ("sin", "cos", "tan"):
            v = _device(ctx, name, np.array([inf, -inf, nan, 0.0, -0.0], dtype=dt))
            assert np.all(np.isnan(v[:3]))
            if name != "cos":
                assert v[3] == 0 and v[4] == 0 and np.signbit(v[4])  # odd functions keep -0.0
            else:
                assert v[3] == 1 and v[4] == 1
        tiny = np.array([np.finfo(dt).tiny, np.finfo(dt).tiny / 4, -np.finfo(dt).tiny / 4], dtype=dt)
        for name in ("sin", "tan"):
            assert np.array_equal(_device(ctx, name, tiny), tiny)  # sin x = x for subnormal / tiny x


def test_device_float32_exp_bits_equal_oracle(ctx, oracle):
    """The packed device exp (srhip_eval_impl.h expf2_dev) returns the oracle's srm_expf bits on 16.7M
    inputs: every 256th bit pattern of the whole float range (all exponents, both signs, NaN / Inf)."""
    x = (np.arange(0, 2**32, 256, dtype=np.uint64).astype(np.uint32)).view(np.float32)
    got = _device(ctx, "exp", x)
    ref = oracle.srm("exp", x)
    nan = np.isnan(x)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), ref[~nan].view(np.uint32))


def test_device_float32_trig_bits_equal_oracle(ctx, oracle):
    """Device Float32 sin / cos (no per-row range select: one max |x| per lane decides whether the
    scalar path redoes the large / Inf / NaN rows) return the oracle's srm_sinf / srm_cosf bits on
    every 256th bit pattern of the float range."""
    x = (np.arange(0, 2**32, 256, dtype=np.uint64).astype(np.uint32)).view(np.float32)
    for name in ("sin", "cos"):
        got = _device(ctx, name, x)
        ref = oracle.srm(name, x)
        nan = np.isnan(ref)
        assert np.array_equal(np.isnan(got), nan), name
        assert np.array_equal(got[~nan].view(np.uint32), ref[~nan].view(np.uint32)), name


def _div_operands(n):
    """Division operand pairs: whole tiles inside the in-range fast path (|n|, |d| in [2^-40, 2^40]),
    whole tiles of arbitrary bit patterns (zeros, subnormals, Inf, NaN, huge), and tiles that mix one
    stray value into in-range rows (the wave falls back to the full division)."""
    def inrange(k):
        return (RNG.choice([-1, 1], k) * 2.0 ** RNG.uniform(-40, 40, k)).astype(np.float32)

    def anybits(k):
        return RNG.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32).view(np.float32)

    q = n // 4
    a = np.concatenate([inrange(q), anybits(q), inrange(q), inrange(q)])
    b = np.concatenate([inrange(q), anybits(q), inrange(q), inrange(q)])
    stray = np.array([0.0, -0.0, np.inf, np.nan, 1e-41, 3e38, 2.0**41, 2.0**-41], dtype=np.float32)
    pos = 2 * q + RNG.choice(q, 64, replace=False)
    a[pos[:32]] = RNG.choice(stray, 32)
    b[pos[32:]] = RNG.choice(stray, 32)
    a[3 * q:3 * q + 8], b[3 * q:3 * q + 8] = 2.0**40, 2.0**-40   # the range boundaries themselves
    a[3 * q + 8:3 * q + 16], b[3 * q + 8:3 * q + 16] = -2.0**-40, -2.0**40
    return a, b


def test_device_float32_division_bits_equal_ieee(ctx):
    """Float32 `/` (srhip_eval_impl.h div_rows: the range-free division for waves whose operands are all in
    [2^-40, 2^40], the full v_div_scale / v_div_fixup sequence otherwise) is IEEE division bit for bit
    (numpy's float32 division) in every instruction form: A / X, X / A, A / c, c / A, A / S, S / A."""
    import srhip

    n = 1 << 20
    a, b = _div_operands(n)
    one = np.ones(n, dtype=np.float32)
    X = np.stack([a, b, one])
    opts = srhip.Options(binary_operators=("+", "-", "*", "/"), unary_operators=())
    x1, x2, x3 = srhip.Node("x1"), srhip.Node("x2"), srhip.Node("x3")
    c = np.float32(0.3716)
    trees = [x1 / x2,                      # A / X
             x1 / (x2 * x3),               # X / A
             x1 / srhip.Node(val=c),       # A / c
             srhip.Node(val=c) / x2,       # c / A
             (x1 * x3) / (x2 * x3),        # S / A or A / S
             (x2 * x3) / ((x1 * x3) * x3)]
    refs = [a / b, a / b, a / c, c / b, a / b, b / a]
    nodes, offs = srhip.flatten(trees, opts, np.float32)
    prog = srhip.Program(ctx, nodes, offs, opts, np.float32)
    pred, _ = prog.eval_predict(srhip.DeviceDataset(ctx, X))
    for t, ref in enumerate(refs):
        got = pred[t]
        nan = np.isnan(ref)
        assert np.array_equal(np.isnan(got), nan), t
        bad = np.nonzero(got[~nan].view(np.uint32) != ref[~nan].view(np.uint32))[0]
        assert len(bad) == 0, (t, len(bad), a[~nan][bad[:4]], b[~nan][bad[:4]], got[~nan][bad[:4]], ref[~nan][bad[:4]])
