"""The three reference preprocessors (PipelineMap.scala:67 valid list):

* ``StandardScaler``     running mean/variance (Chan et al. parallel merge of the batch
                         moments into the running moments), transform (x − μ)/σ
* ``MinMaxScaler``       running per-feature min/max, transform (x − min)/(max − min)
* ``PolynomialFeatures`` degree-d monomial expansion of the dense features (default 2):
                         [x, x_i·x_j (i ≤ j), ...]

They act on the dense block ``batch.num`` (numerical ∥ discrete features) of a micro-batch;
hashed categorical slots pass through untouched. Statistics are updated with the batch
*before* it is transformed (micro-batch form of the per-point update-then-transform).
On GPU the column moments and the transform run as hand-written HIP kernels
(csrc/kernels/preprocess.hip); the CPU path uses the identical math in PyTorch.
"""
from __future__ import annotations

import itertools

import torch

from omldm_amd.api.batch import HashedBatch
from omldm_amd.ops import preprocess as P


class Preprocessor:
    NAME = "Preprocessor"

    def __init__(self, hyper: dict | None, device="cpu"):
        self.hyper = dict(hyper or {})
        self.device = torch.device(device)

    def out_dim(self, d: int) -> int:
        return d

    def fit_transform(self, x: torch.Tensor, train: bool) -> torch.Tensor:
        raise NotImplementedError

    def __call__(self, batch: HashedBatch, train: bool = True) -> HashedBatch:
        if batch.B == 0:
            num = torch.zeros((0, self.out_dim(batch.dn)), dtype=torch.float32,
                              device=batch.num.device)
            return HashedBatch(num, batch.cat, batch.y, batch.raw, batch.cat_span)
        # the categorical slots pass through untouched, in their wire format (cat_span)
        return HashedBatch(self.fit_transform(batch.num.float().contiguous(), train), batch.cat,
                           batch.y, batch.raw, batch.cat_span)

    def state_dict(self) -> dict:
        return {}

    def load_state_dict(self, sd: dict) -> None:
        pass

    def to_obj(self) -> dict:
        return {"name": self.NAME, "hyperParameters": self.hyper, "parameters": {
            k: (v.tolist() if torch.is_tensor(v) else v) for k, v in self.state_dict().items()}}

    # dtype of each list-valued parameter when imported (to_obj → Create warm start)
    PARAM_DTYPES: dict = {}

    def load_parameters(self, params: dict) -> None:
        """Warm start from ``to_obj()["parameters"]`` (a Create's preProcessors entry)."""
        sd = {}
        for k, v in params.items():
            if isinstance(v, list):
                sd[k] = torch.tensor(v, dtype=self.PARAM_DTYPES.get(k, torch.float32))
            else:
                sd[k] = v
        self.load_state_dict({**self.state_dict(), **sd})


class StandardScaler(Preprocessor):
    NAME = "StandardScaler"
    PARAM_DTYPES = {"mean": torch.float64, "m2": torch.float64}

    def __init__(self, hyper=None, device="cpu"):
        super().__init__(hyper, device)
        self.count = 0.0
        self.mean = None
        self.m2 = None

    def fit_transform(self, x, train):
        if self.mean is None:
            self.mean = torch.zeros(x.shape[1], dtype=torch.float64, device=x.device)
            self.m2 = torch.zeros_like(self.mean)
        if train:
            self.count = P.welford_update(x, self.count, self.mean, self.m2)
        return P.standardize(x, self.mean, self.m2, self.count)

    def state_dict(self):
        return {"count": self.count, "mean": self.mean, "m2": self.m2}

    def load_state_dict(self, sd):
        self.count = float(sd["count"])
        self.mean = sd["mean"].to(self.device) if sd["mean"] is not None else None
        self.m2 = sd["m2"].to(self.device) if sd["m2"] is not None else None


class MinMaxScaler(Preprocessor):
    NAME = "MinMaxScaler"

    def __init__(self, hyper=None, device="cpu"):
        super().__init__(hyper, device)
        self.lo = None
        self.hi = None

    def fit_transform(self, x, train):
        if self.lo is None:
            self.lo = torch.full((x.shape[1],), float("inf"), device=x.device)
            self.hi = torch.full((x.shape[1],), float("-inf"), device=x.device)
        if train:
            P.minmax_update(x, self.lo, self.hi)
        return P.minmax_scale(x, self.lo, self.hi)

    def state_dict(self):
        return {"min": self.lo, "max": self.hi}

    def load_state_dict(self, sd):
        self.lo = sd["min"].to(self.device) if sd["min"] is not None else None
        self.hi = sd["max"].to(self.device) if sd["max"] is not None else None


class PolynomialFeatures(Preprocessor):
    NAME = "PolynomialFeatures"

    def __init__(self, hyper=None, device="cpu"):
        super().__init__(hyper, device)
        self.degree = int(self.hyper.get("degree", 2))
        self._pairs = {}

    def out_dim(self, d: int) -> int:
        return sum(len(list(itertools.combinations_with_replacement(range(d), k)))
                   for k in range(1, self.degree + 1))

    def _index(self, d: int, device) -> torch.Tensor:
        key = (d, str(device))
        if key not in self._pairs:
            combos = [c for k in range(2, self.degree + 1)
                      for c in itertools.combinations_with_replacement(range(d), k)]
            width = self.degree
            idx = torch.full((len(combos), width), -1, dtype=torch.int32)
            for r, c in enumerate(combos):
                idx[r, : len(c)] = torch.tensor(c, dtype=torch.int32)
            self._pairs[key] = idx.to(device)
        return self._pairs[key]

    def fit_transform(self, x, train):
        return P.poly_expand(x, self._index(x.shape[1], x.device))

    def pair_index(self, d: int, device) -> torch.Tensor:
        """int32 [np, 2] (a, b) of the degree-2 products appended after the d inputs (the
        fused learners' form of this map; degree 2 only)."""
        assert self.degree == 2
        return self._index(d, device)


PREPROCESSORS = {c.NAME: c for c in (StandardScaler, MinMaxScaler, PolynomialFeatures)}


def make_preprocessor(name: str, hyper: dict | None, device) -> Preprocessor:
    return PREPROCESSORS[name](hyper, device)
