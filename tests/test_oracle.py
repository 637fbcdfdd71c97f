"""The C oracle's restated loss families (test infrastructure: oracle/sr_oracle.c) against the
Python mirror's independent numpy forms."""
import numpy as np

from conftest import ROOT  # noqa: F401  (puts the package and the oracle on sys.path)

def test_oracle_margin_losses_vs_numpy(oracle):
    """The oracle's LossFunctions margin losses (sr_oracle.c margin_f64, restated from LossFunctions.jl
    0.11 src/losses/margin.jl) == the Python mirror's numpy forms (srhip/losses.py) on a feature-leaf
    tree (prediction = x1) with +-1 targets -- two independent restatements of the published
    definitions (the package itself is not in the container: parity with it is unpinned)."""
    import srhip as sr

    opts = sr.Options(binary_operators=("+",), unary_operators=())
    nodes, offs = sr.flatten([sr.Node("x1")], opts, np.float64)
    rng = np.random.default_rng(3)
    X = rng.uniform(-3, 3, (1, 4000))
    y = np.where(rng.standard_normal(4000) > 0, 1.0, -1.0)
    for L in (sr.ZeroOneLoss(), sr.PerceptronLoss(), sr.LogitMarginLoss(), sr.L1HingeLoss(), sr.L2HingeLoss(),
              sr.SmoothedL1HingeLoss(0.6), sr.ModifiedHuberLoss(), sr.L2MarginLoss(), sr.ExpLoss(), sr.SigmoidLoss(),
              sr.DWDMarginLoss(1.5)):
        le, _, ok, _ = oracle.eval_loss_batch(nodes, offs, opts.binop_codes, opts.unaop_codes, X, y, None, L.kind, L.p0)
        ref = float(np.mean(L(X[0], y)))
        assert ok[0] and abs(le[0] - ref) <= 1e-12 * max(1.0, abs(ref)), (type(L).__name__, le[0], ref)
