"""Learner interface shared by all eight reference learners (+ extensions).

Reference: mlAPI learners are driven through ``MLPipeline.pipePoint`` (fit one point)
and expose parameters / hyper-parameters / data-structure maps in query responses
(omldm/network/FlinkNetwork.scala:151-240). Here a learner is driven
one *micro-batch round* at a time and keeps all of its state in device tensors:

* ``fit(batch, ctx)`` trains on a micro-batch (virtual spokes inside when the learner
  supports them) and returns device-side round statistics (no host sync);
* ``state_vector()`` is the flat fp32 view that the synchronisation protocols ship over
  RCCL; ``merge_mode`` says how worker states combine: ``"mean"`` (model averaging) or
  ``"sum"`` (additive sufficient statistics: ORR, K-means);
* ``predict``/``evaluate`` serve forecasts and holdout scoring.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch


@dataclass
class RoundContext:
    spokes: int = 1          # virtual spokes on this rank for this round
    inv_p: float = 1.0       # 1 / (number of workers the round's delta is averaged over)
    fused_delta: bool = False  # leave the round delta in the sync buffer (Synchronous fast path)
    # pipelined sync (learners with supports_reduce_parts): the delta reduce runs in
    # ``reduce_parts`` launches and ``on_reduce_part(k, lo, hi)`` is called right after
    # part k is enqueued, with the slice [lo, hi) of the sync buffer it completes — the
    # protocol starts that slice's collective while the next part reduces
    reduce_parts: int = 1
    on_reduce_part: Callable[[int, int, int], None] | None = None


class Learner:
    NAME = "Learner"
    TASK = "classification"  # classification | regression | clustering
    merge_mode = "mean"
    supports_fused_delta = False
    supports_reduce_parts = False

    def reduce_parts_apply(self, batch, ctx) -> bool:
        """Whether this round's reduce really runs in key-range parts (the pipelined sync
        starts each part's collective as soon as it is final); False when the round's kernel
        completes the accumulator only at its end, so a parts split would be a no-op."""
        return self.supports_reduce_parts

    def __init__(self, hyper: dict | None, space: FeatureSpace, device="cpu"):
        self.hyper = dict(hyper or {})
        self.space = space
        self.device = torch.device(device)
        # device-side running counters: loss_sum, n, mistakes, sq_err, -, overflow, -, -
        # fp64: kernels add per-round fp32 partials into them, and an fp32 total stops
        # counting once it passes 2^24..2^31 (integer increments round away)
        self.cum = torch.zeros(8, dtype=torch.float64, device=self.device)

    # ---------------------------------------------------------------- training
    def fit(self, batch: HashedBatch, ctx: RoundContext) -> None:
        raise NotImplementedError

    def apply_delta(self) -> None:
        """Fold the (all-reduced) fused round delta into the model."""

    def delta_buffer(self) -> torch.Tensor | None:
        return None

    # ------------------------------------------------------ protocol state view
    def state_vector(self) -> torch.Tensor:
        raise NotImplementedError

    def load_state_vector(self, v: torch.Tensor) -> None:
        self.state_vector().copy_(v)
        self.on_state_loaded()

    def on_state_loaded(self) -> None:
        pass

    def num_params(self) -> int:
        return int(self.state_vector().numel())

    # ---------------------------------------------------------------- inference
    def predict(self, batch: HashedBatch) -> torch.Tensor:
        raise NotImplementedError

    def evaluate(self, batch: HashedBatch) -> tuple[torch.Tensor, torch.Tensor, int]:
        """(loss_sum, score_sum, n) on labelled points as device scalars."""
        raise NotImplementedError

    # ---------------------------------------------------------------- API maps
    def hyper_parameters(self) -> dict:
        """The user-visible hyper-parameters (engine-internal ``_``-keys left out)."""
        return {k: v for k, v in self.hyper.items() if not str(k).startswith("_")}

    # hyper-parameters that fix the model's shape: an Update may not change them on a
    # live pipeline (it is dropped and counted, like any invalid request)
    STRUCTURAL: tuple = ()

    def structural_values(self) -> dict:
        """The shape-fixing values IN USE (not what Create happened to spell out), keyed
        like the hyper-parameters, in the normalised form of ``_norm_structural``."""
        return {}

    @staticmethod
    def _norm_structural(k: str, v):
        """One comparable form per structural value: '[8, 8]' / [8, 8] / (8, 8) → (8, 8),
        '4' / 4 / 4.0 → 4, anything else → its string."""
        if isinstance(v, str):
            t = v.strip()
            if t.startswith("[") and t.endswith("]"):
                try:
                    return tuple(int(x) for x in t[1:-1].split(",") if x.strip())
                except ValueError:
                    return t
            try:
                f = float(t)
                return int(f) if f == int(f) else f
            except ValueError:
                return t
        if isinstance(v, (list, tuple)):
            try:
                return tuple(int(x) for x in v)
            except (TypeError, ValueError):
                return tuple(v)
        if isinstance(v, bool):
            return v
        if isinstance(v, (int, float)):
            return int(v) if float(v) == int(v) else float(v)
        return str(v)

    def update_hyper(self, hyper: dict) -> None:
        """Apply an Update atomically: the merged hyper-parameters are validated and the
        derived settings rebuilt first; on any error the learner is left exactly as it
        was (nothing of a rejected Update is applied), and the error propagates so the
        engine drops and counts the request."""
        hyper = dict(hyper or {})
        cur = self.structural_values()
        for k in self.STRUCTURAL:
            if k in hyper and k in cur and \
                    self._norm_structural(k, hyper[k]) != self._norm_structural(k, cur[k]):
                raise ValueError(f"{self.NAME}: {k} cannot change on a live pipeline")
        saved = dict(self.__dict__)  # shallow: _retune rebinds, never mutates in place
        self.hyper = {**self.hyper, **hyper}
        try:
            self._retune()
        except Exception:
            self.__dict__.clear()
            self.__dict__.update(saved)
            raise

    def _retune(self) -> None:
        """Re-read the tunable hyper-parameters after an Update or a restore (learning
        rates, margins, split thresholds); the base learner has none. Must rebind
        attributes rather than mutate tensors in place (update_hyper rolls back by
        restoring the attribute dict)."""

    def parameters_map(self) -> dict:
        """The learner's COMPLETE parameters as JSON-able lists/scalars — the reference's
        only portable model format (QueryResponse ``learner.parameters``, bucketed by
        10,000 on the wire, FlinkNetwork.scala:48-240). ``load_parameters`` of a fresh
        learner with the same hyper-parameters reproduces the model exactly."""
        return {}

    def load_parameters(self, params: dict) -> None:
        """Warm start from ``parameters_map()`` output (a Create request's
        ``learner.parameters``, bucketed keys already merged)."""
        raise ValueError(f"{self.NAME}: no importable parameters")

    @staticmethod
    def _vec(params: dict, key: str, n: int | None = None) -> torch.Tensor:
        v = params[key]
        t = torch.as_tensor(v if isinstance(v, (list, tuple)) else [v], dtype=torch.float64)
        if n is not None and t.numel() != n:
            raise ValueError(f"parameter {key!r}: {t.numel()} values, expected {n}")
        return t

    def data_structure(self) -> dict:
        return {"learner": self.NAME, "task": self.TASK, "nParams": self.num_params()}

    # ---------------------------------------------------------------- checkpoint
    def state_dict(self) -> dict:
        return {"state": self.state_vector().detach().cpu().clone(), "cum": self.cum.cpu().clone(),
                "hyper": dict(self.hyper)}

    def load_state_dict(self, sd: dict) -> None:
        self.hyper.update(sd.get("hyper", {}))
        self._retune()  # the restored (possibly Updated) settings, not Create's
        self.load_state_vector(sd["state"].to(self.device))
        if "cum" in sd:
            self.cum.copy_(sd["cum"].to(self.device, torch.float64))

    def running_totals(self) -> dict:
        c = self.cum.tolist()
        return {"loss_sum": c[0], "fitted": int(c[1]), "mistakes": c[2], "sq_err": c[3],
                "overflow": int(c[5])}


def hp_float(h: dict, key: str, default: float) -> float:
    v = h.get(key, default)
    try:
        return float(v)
    except (TypeError, ValueError):
        return default


def hp_int(h: dict, key: str, default: int) -> int:
    v = h.get(key, default)
    try:
        return int(v)
    except (TypeError, ValueError):
        return default
