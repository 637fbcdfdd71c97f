"""Dataset{T,L} mirror (reference src/Dataset.jl:53-82, constructor :98-225).

X is (nfeatures, n) (FEATURE_DIM = 1, BATCH_DIM = 2 in src/ProgramConstants.jl:4-5).  The device
copy is made lazily, once per context, and reused by every evaluation on this dataset: that is
the "dataset stays device-resident in HBM" half of the design.
"""
from __future__ import annotations

import numpy as np


class Dataset:
    def __init__(self, X, y=None, weights=None, loss_type=None, variable_names=None, extra=None, X_units=None,
                 y_units=None):
        X = np.asarray(X)
        if X.ndim == 1:
            X = X.reshape(1, -1)
        if X.dtype not in (np.float32, np.float64, np.int32):
            X = X.astype(np.float64)
        self.X = X
        self.nfeatures, self.n = X.shape
        T = X.dtype.type
        self.y = None if y is None else np.asarray(y, dtype=X.dtype).reshape(-1)
        self.weights = None if weights is None else np.asarray(weights, dtype=X.dtype).reshape(-1)
        self.weighted = self.weights is not None
        if self.y is not None and len(self.y) != self.n:
            raise ValueError("y must have n entries")
        if self.weighted and len(self.weights) != self.n:
            raise ValueError("weights must have n entries")
        # avg_y (src/Dataset.jl:155-163), computed in T as the reference does
        if self.y is None:
            self.avg_y = None
        elif self.weighted:
            self.avg_y = T(np.sum(self.y * self.weights, dtype=X.dtype) / np.sum(self.weights, dtype=X.dtype))
        else:
            self.avg_y = T(np.sum(self.y, dtype=X.dtype) / T(self.n)) if X.dtype != np.int32 else \
                np.float64(np.sum(self.y, dtype=np.int64)) / self.n
        # loss type L (src/Dataset.jl:164-168): default T; Int32 data evaluates losses in Float64
        if loss_type is None:
            loss_type = np.float64 if X.dtype == np.int32 else X.dtype
        self.loss_type = np.dtype(loss_type)
        self.variable_names = variable_names or [f"x{i + 1}" for i in range(self.nfeatures)]
        self.extra = extra or {}
        self.use_baseline = True
        self.baseline_loss = self.loss_type.type(1)
        # units (src/Dataset.jl:170-193): y_units without X_units makes every feature dimensionless
        from .units import get_units

        self.y_units = get_units(y_units)
        self.X_units = get_units(X_units, self.nfeatures)
        if self.X_units is None and self.y_units is not None:
            self.X_units = get_units(["1"] * self.nfeatures)
        self._dev = {}

    def has_units(self) -> bool:
        return self.X_units is not None

    def device(self, ctx):
        """The DeviceDataset for `ctx` (uploaded on first use)."""
        from .device import DeviceDataset

        key = (id(ctx), ctx.device)
        d = self._dev.get(key)
        # a cached copy keeps its Context object alive (so the id is not reused), but the
        # context may have been closed explicitly: upload again then
        if d is not None and (d.ctx is not ctx or d.handle is None or ctx.handle is None):
            d = None
        if d is None:
            d = self._dev[key] = DeviceDataset(ctx, self.X, self.y, self.weights)
        return d

    def release_device(self, ctx) -> None:
        """Free the device copy held for `ctx` (before closing that context)."""
        d = self._dev.pop((id(ctx), ctx.device), None)
        if d is not None:
            d.close()
