"""Online linear learners on hashed features: PA, SVM, RegressorPA (+ LogisticRegression).

Reference learner names come from the request validator
(omldm/utils/parsers/requestStream/PipelineMap.scala:68); the update rules are the
published Passive-Aggressive family (Crammer et al. 2006) — SURVEY.md Appendix D:

* ``PA``          binary hinge, τ = ℓ/‖x‖² (variant "PA"), min(C, ℓ/‖x‖²) ("PA-I"),
                  ℓ/(‖x‖² + 1/(2C)) ("PA-II"); default PA-I.
* ``SVM``         online linear SVM: hinge loss + L2 (``lambda`` shrink per step) with the
                  PA-I step (BASELINE.json config 1: "Online linear SVM (PA-I)");
                  ``variant: "Pegasos"`` (PA and SVM) selects Pegasos SGD instead (SURVEY
                  Appendix D): at the spoke's step T, η = 1/(λT) and
                  w ← (1 − 1/T)·w + η·y·x·[y·w·x < 1]; T counts each spoke's rows from
                  ``t0`` + 1 (default t0 = 1, so σ never reaches 0; λ defaults to 1e-4).
* ``RegressorPA`` ε-insensitive loss, same τ family, update sign(y − w·x)·τ·x.
* ``LogisticRegression`` (extension, BASELINE.json config 2): SGD on the log loss.

A round is S virtual spokes, each an exact sequential learner on its R-row shard. On a GPU
every rule — the PA family, RegressorPA, logistic SGD, SVM's L2 shrink, Pegasos, bf16
models — runs the v3 table scan (csrc/kernels/linear_scan3.hip: chunk Grams on the matrix
cores, one scan workgroup per spoke with its updates in an LDS slot table; the shrinking
rules carry the spoke's model scale σ through the chain) on the raw wire and on the
engine's field-aware hashed batches (bench/learners.py --preset p16: 228–277 M ex/s at
16 spokes, profiles/round6/learners_p16.json). What v3 does not take falls back, logged:
raw batches of an unsupported shape without a shrink to v1 (csrc/kernels/linear_seq.hip);
non-field-aware hashed batches, more than 32 categorical fields or R > 8192 rows per
spoke to the spoke-table round (csrc/kernels/linear_spoke.hip: per-spoke LDS delta tables
spilling to HBM, spoke_table.h, ≈1.2 M ex/s).
"""
from __future__ import annotations

import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch, RawBatch
from omldm_amd.models.base import Learner, RoundContext, hp_float, hp_int
from omldm_amd.ops import linear as L

_VARIANTS = {"PA": L.PA, "PA-I": L.PA1, "PA1": L.PA1, "PA-II": L.PA2, "PA2": L.PA2}


class LinearLearner(Learner):
    NAME = "Linear"
    RULE = L.RULE_HINGE
    DEFAULT_VARIANT = "PA-I"
    supports_fused_delta = True
    supports_reduce_parts = True

    def __init__(self, hyper: dict | None, space: FeatureSpace, device="cpu"):
        super().__init__(hyper, space, device)
        self.dim = space.dim
        self.w = torch.zeros(self.dim, dtype=torch.float32, device=self.device)
        self.w16 = None
        self.dacc = torch.zeros(self.dim + 2, dtype=torch.float32, device=self.device)
        # raw-wire rounds on the GPU: per-spoke fp32 replicas [S, dim] (linear_seq.hip),
        # equal to w between rounds; invalidated whenever w changes outside a round
        self.replicas = None
        self._rep_valid = False
        self._seq_pending = False
        self._configure()

    def _configure(self) -> None:
        h = self.hyper
        variant = str(h.get("variant", self.DEFAULT_VARIANT))
        pegasos = variant.lower() == "pegasos" and self.RULE == L.RULE_HINGE
        self.rule = L.LinearRule(
            rule=L.RULE_PEGASOS if pegasos else self.RULE,
            variant=_VARIANTS.get(variant, L.PA1),
            C=hp_float(h, "C", 1.0),
            eps=hp_float(h, "epsilon", 0.1),
            lr=hp_float(h, "learningRate", 0.1),
            lam=hp_float(h, "lambda", 1e-4 if pegasos else 0.0),
            bias=bool(h.get("bias", True)),
        )
        if pegasos and not self.rule.lam > 0:
            raise ValueError("Pegasos needs lambda > 0")
        self.t0 = max(1, hp_int(h, "t0", 1))
        if not hasattr(self, "steps"):
            self.steps = 0  # rows per spoke trained in earlier rounds (the Pegasos clock)
        self.log2cap = hp_int(h, "tableLog2", 0)  # 0: auto (ops/linear.py:auto_log2cap)
        self.ablate = hp_int(h, "_ablate", 0)  # timing diagnostics only
        self.chunk = hp_int(h, "chunk", 8)      # rows staged per software-pipeline step
        want16 = str(h.get("modelDtype", "fp32")).lower() in ("bf16", "bfloat16")
        if want16 and self.w16 is None:
            self.w16 = self.w.to(torch.bfloat16)
        elif not want16:
            self.w16 = None

    def _retune(self) -> None:
        self._configure()

    # ---------------------------------------------------------- model store rows
    def attach(self, row: torch.Tensor) -> None:
        """Re-point the fp32 weights at a row of the HBM model store (engine/model_store.py);
        ``row`` already holds the current weights."""
        self.w = row
        self._rep_valid = False

    def detach(self) -> None:
        self.w = self.w.clone()
        self._rep_valid = False

    def vector_bias(self) -> tuple[torch.Tensor, float]:
        """The reference's ``VectorBias(weights, bias)`` view: the
        intercept lives in the reserved last slot of the flat weight vector."""
        return self.w[: self.dim - 1], float(self.w[self.dim - 1]) if self.rule.bias else 0.0

    # ---------------------------------------------------------------- training
    def _wread(self) -> torch.Tensor:
        return self.w16 if self.w16 is not None else self.w

    def seq_capable(self, batch=None, ctx: RoundContext | None = None) -> bool:
        """Raw-wire rounds run the exact sequential Gram-scan kernels (PA family, RegressorPA,
        logistic SGD; v3 or v1). The shrinking rules (L2 λ > 0, Pegasos) and bf16 models have
        only the v3 form: on a GPU, where the v3 scan takes ``batch`` (None: the caller checks
        the shape). Everything else hashes the batch and takes the spoke-table round."""
        if not L.shrinks(self.rule) and self.w16 is None:
            return self.rule.rule in L.SEQ_RULES
        if not (self.w.is_cuda and L.SEQ_KERNEL == "scan3"):
            return False
        if batch is None:
            return True
        R, _ = self._seq_geometry(batch.B, ctx) if ctx is not None else (batch.B, 1)
        return bool(batch.B) and L.scan3_eligible(batch, R, self.rule.bias)

    def reduce_parts_apply(self, batch, ctx: RoundContext) -> bool:
        """The spoke-table round reduces its tables in key-range parts; the v3 table scan
        completes the accumulator only at its round end (no part is final earlier), so a
        batch it takes runs one reduce and one collective."""
        if not self.supports_reduce_parts:
            return False
        if isinstance(batch, RawBatch):
            return not self.seq_capable(batch, ctx)
        return self.group_key(batch, ctx) is None

    @staticmethod
    def _seq_geometry(B: int, ctx: RoundContext) -> tuple[int, int]:
        S = max(1, int(ctx.spokes))
        R = max(1, -(-B // S)) if B else 1
        S = max(1, -(-B // R)) if B else S
        return R, S

    def _slots_scan_eligible(self, batch, ctx: RoundContext | None = None) -> bool:
        """The engine's field-aware hashed batches train through the v3 table scan, which
        reads their compact int16 slots as they are; other hashed batches take the
        spoke-table round."""
        if not (type(batch) is HashedBatch and batch.cat_span > 0 and self.w.is_cuda
                and self.seq_capable() and batch.B > 0 and 0 < batch.dc
                and L.SEQ_KERNEL == "scan3"
                and self.space.dn + batch.dc * batch.cat_span <= self.dim - 1):
            return False
        R, _ = self._seq_geometry(batch.B, ctx) if ctx is not None else (batch.B, 1)
        return bool(L.scan3_fits(batch.dn, batch.dc, R, self.rule.bias))

    def _fit_slots(self, batch: HashedBatch, ctx: RoundContext) -> None:
        num, y = batch.num.float().contiguous(), batch.y.float().contiguous()
        R, _ = self._seq_geometry(batch.B, ctx)
        rb = RawBatch(num, batch.cat.contiguous(), y, span=batch.cat_span, cbase=self.space.dn)
        # a v3 prep made ahead for this batch (engine/job.py route stream, or the first
        # pipeline of the tick that trains on it; ops.linear checks that it matches)
        rb.prep = getattr(batch, "prep", None)
        assert L.scan3_eligible_compact(rb, R, self.rule.bias, self.dim), "v3 shape check"
        self._fit_raw(rb, ctx, hashed=True)
        batch.prep = rb.prep

    def _fit_raw(self, batch: RawBatch, ctx: RoundContext, hashed: bool = False) -> None:
        B = batch.B
        R, S = self._seq_geometry(B, ctx)
        on_gpu = self.w.is_cuda
        # v3 (the table scan) keeps no dense replicas: its round end sums the spokes'
        # updates from the sorted occurrence lists; v1 / v2 average [S, dim] replicas
        use_rep = on_gpu and not (B and L.scan3_eligible(batch, R, self.rule.bias))
        if use_rep:
            if self.replicas is None or self.replicas.shape[0] < S:
                self.replicas = torch.empty((S, self.dim), dtype=torch.float32, device=self.device)
                self._rep_valid = False
            if not self._rep_valid:
                L.linear_seq_broadcast(self.w, self.replicas)
                self._rep_valid = True
        parts = max(1, int(ctx.reduce_parts)) if ctx.on_reduce_part is not None else 1
        if B:
            self.rule.tbase = float(self.t0 + 1 + self.steps)  # Pegasos' step clock
            L.linear_seq_round(self._wread(), batch, R, S, self.dacc, self.rule, ctx.inv_p,
                               cum=self.cum, replicas=self.replicas if use_rep else None,
                               parts=parts, on_part=ctx.on_reduce_part, hashed=hashed)
            self.steps += R
        else:
            self.dacc[self.dim:].zero_()
            if ctx.on_reduce_part is not None:  # still join every collective of the round
                for k in range(parts):
                    ctx.on_reduce_part(k, *L.part_bounds(self.dim, k, parts, self.dacc.is_cuda))
        self._seq_pending = use_rep
        if not ctx.fused_delta:
            self.apply_delta()

    # ------------------------------------------------------ several pipelines
    def group_key(self, batch, ctx: RoundContext):
        """Learners whose rounds on ``batch`` can share ONE v3 launch (same prep, same rule
        family and variant, no shrink, fp32): a key, or None when this one cannot."""
        if not (self.w.is_cuda and self.seq_capable() and batch.B > 0):
            return None
        if isinstance(batch, RawBatch):
            rb = batch
            R, _ = self._seq_geometry(batch.B, ctx)
            if not L.scan3_eligible(rb, R, self.rule.bias):
                return None
        else:
            b = batch.spoke_padded(max(1, int(ctx.spokes)))
            if not self._slots_scan_eligible(b, ctx):
                return None
        r = self.rule
        r.tbase = float(self.t0 + 1 + self.steps)  # (Pegasos: the prep depends on the clock)
        # (logistic: lr·y is folded into the prep's Gram columns, so only equal learning
        # rates share a prep — ops.linear._s3_key)
        return (self.dim, r.rule, r.variant, r.bias, r.C if r.variant == L.PA2 else None,
                L._s3_shrink(r), self.w16 is not None,
                float(r.lr) if r.rule == L.RULE_LOGISTIC else None)

    def prepare_ahead(self, batch: HashedBatch, ctx: RoundContext, stream) -> bool:
        """Make the v3 prep of this learner's round on ``batch`` now, on ``stream``, and
        attach it to the spoke-padded batch its ``fit`` will use (engine/job.py: the next
        tick's route + prep run beside the current round). False: no v3 round here."""
        if self.group_key(batch, ctx) is None:
            return False
        b = batch.spoke_padded(max(1, int(ctx.spokes)))
        R, S = self._seq_geometry(b.B, ctx)
        rb = RawBatch(b.num.float().contiguous(), b.cat.contiguous(), b.y.float().contiguous(),
                      span=b.cat_span, cbase=self.space.dn)
        key = L._s3_key(rb, R, S, self.dim, self.rule.bias, self.rule)
        if isinstance(b.prep, L.Scan3Prep) and b.prep.key == key:
            return True
        b.prep = L.linear_scan3_prepare(rb, R, S, self.dim, bool(self.rule.bias), self.rule,
                                        slot=L._s3_slot_for(key, self.w.device), stream=stream,
                                        hashed=True)
        return True

    @staticmethod
    def fit_group(learners: list, batch, ctx: RoundContext) -> None:
        """One round of every learner in ``learners`` (equal ``group_key``) on ``batch`` in
        one launch (ops.linear.linear_scan3_round_multi) — each learner ends exactly as its
        own ``fit`` would leave it."""
        first = learners[0]
        hashed = False
        if isinstance(batch, RawBatch):
            rb = batch
        else:
            b = batch.spoke_padded(max(1, int(ctx.spokes)))
            rb = RawBatch(b.num.float().contiguous(), b.cat.contiguous(), b.y.float().contiguous(),
                          span=b.cat_span, cbase=first.space.dn)
            rb.prep = getattr(b, "prep", None)
            hashed = True
        R, S = first._seq_geometry(rb.B, ctx)
        for lr in learners:
            lr.rule.tbase = float(lr.t0 + 1 + lr.steps)
        step = L.scan3_max_pipes()
        for i in range(0, len(learners), step):
            grp = learners[i:i + step]
            L.linear_scan3_round_multi([lr._wread() for lr in grp], rb, R, S,
                                       [lr.dacc for lr in grp],
                                       [lr.rule for lr in grp], ctx.inv_p,
                                       [lr.cum for lr in grp], hashed=hashed)
        if not isinstance(batch, RawBatch):
            batch.prep = rb.prep
        for lr in learners:
            lr._seq_pending = False
            lr.steps += R
        if not ctx.fused_delta:  # the models averaged in one launch
            LinearLearner.apply_delta_group(learners)

    def fit(self, batch: HashedBatch, ctx: RoundContext) -> None:
        if isinstance(batch, RawBatch):
            if self.seq_capable(batch, ctx):
                return self._fit_raw(batch, ctx)
            batch = batch.hashed(self.space)
        # a holdout-routed tick: spoke s trains exactly the rows spoke s routed
        batch = batch.spoke_padded(max(1, int(ctx.spokes)))
        if self._slots_scan_eligible(batch, ctx):
            return self._fit_slots(batch, ctx)
        B = batch.B
        S = max(1, int(ctx.spokes))
        R = max(1, -(-B // S)) if B else 1
        parts = max(1, int(ctx.reduce_parts)) if ctx.on_reduce_part is not None else 1
        if B:
            self.rule.tbase = float(self.t0 + 1 + self.steps)
            L.linear_round(self._wread(), batch, R, S, self.dacc, None, self.rule, ctx.inv_p,
                           self.log2cap, cum=self.cum, ablate=self.ablate, chunk=self.chunk,
                           parts=parts, on_part=ctx.on_reduce_part)
            self.steps += R
        else:
            self.dacc[self.dim:].zero_()  # no workers this round on this rank
            if ctx.on_reduce_part is not None:  # still join every collective of the round
                for k in range(parts):
                    ctx.on_reduce_part(k, *L.part_bounds(self.dim, k, parts, self.dacc.is_cuda))
        if not ctx.fused_delta:
            self.apply_delta()

    def delta_buffer(self) -> torch.Tensor:
        return self.dacc

    @staticmethod
    def apply_delta_group(learners: list) -> None:
        """``apply_delta`` of every learner; the plain averages (equal dimension) in one
        launch."""
        plain = [lr for lr in learners if not (lr._seq_pending and lr.replicas is not None)]
        dims = {int(lr.w.shape[0]) for lr in plain}
        if len(plain) > 1 and len(dims) == 1 and plain[0].w.is_cuda:
            L.linear_apply_multi([lr.w for lr in plain], [lr.w16 for lr in plain],
                                 [lr.dacc for lr in plain])
            for lr in plain:
                lr._rep_valid = False
            rest = [lr for lr in learners if lr not in plain]
        else:
            rest = learners
        for lr in rest:
            lr.apply_delta()

    def apply_delta(self) -> None:
        if self._seq_pending and self.replicas is not None:
            # average + refresh every replica in one pass (they stay equal to w)
            L.linear_seq_apply(self.w, self.replicas, self.dacc)
            self._seq_pending = False
            return
        L.linear_apply(self.w, self.w16, self.dacc)
        self._rep_valid = False

    def state_dict(self) -> dict:
        return {**super().state_dict(), "steps": self.steps}

    def load_state_dict(self, sd: dict) -> None:
        super().load_state_dict(sd)
        self.steps = int(sd.get("steps", self.steps))

    # ------------------------------------------------------------ protocol view
    def state_vector(self) -> torch.Tensor:
        return self.w

    def on_state_loaded(self) -> None:
        self._rep_valid = False
        if self.w16 is not None:
            self.w16.copy_(self.w)

    # ---------------------------------------------------------------- inference
    def decision(self, batch: HashedBatch) -> torch.Tensor:
        return L.linear_predict(self._wread(), batch, bias=self.rule.bias)

    def predict(self, batch: HashedBatch) -> torch.Tensor:
        s = self.decision(batch)
        if self.TASK == "classification":
            return torch.where(s >= 0, 1.0, -1.0)
        return s

    def evaluate(self, batch: HashedBatch):
        s = self.decision(batch)
        y = batch.y
        ok = ~torch.isnan(y)
        n = int(ok.sum().item()) if batch.B else 0
        if self.TASK == "classification":
            ym = (y * s)[ok]
            if self.RULE == L.RULE_LOGISTIC:
                loss = torch.nn.functional.softplus(-ym).sum()
            else:
                loss = torch.clamp(1 - ym, min=0).sum()
            score = (ym > 0).float().sum()
        else:
            e = (y - s)[ok]
            loss = torch.clamp(e.abs() - self.rule.eps, min=0).sum()
            score = (e * e).sum()  # summed squared error → RMSE at the reducer
        return loss, score, n

    # ---------------------------------------------------------------- API maps
    def hyper_parameters(self) -> dict:
        r = self.rule
        names = {L.PA: "PA", L.PA1: "PA-I", L.PA2: "PA-II"}
        variant = "Pegasos" if r.rule == L.RULE_PEGASOS else names[r.variant]
        return {**super().hyper_parameters(), "C": r.C, "variant": variant, "epsilon": r.eps,
                "learningRate": r.lr, "lambda": r.lam, "bias": r.bias}

    def parameters_map(self) -> dict:
        """The reference's VectorBias (weights + intercept): all dim − 1 hashed
        weights (numerical slots first), dense."""
        w = self.w.detach().float().cpu()
        return {"weights": w[: self.dim - 1].tolist(),
                "intercept": float(w[self.dim - 1]) if self.rule.bias else 0.0}

    def load_parameters(self, params: dict) -> None:
        """Dense ``weights`` (≤ dim − 1 values) or sparse ``nonZeroIndices`` /
        ``nonZeroWeights``, plus ``intercept``."""
        w = torch.zeros(self.dim, dtype=torch.float32)
        if "weights" in params and params["weights"] is not None:
            v = self._vec(params, "weights")
            if v.numel() > self.dim - 1:
                raise ValueError(f"{self.NAME}: {v.numel()} weights for a {self.dim}-slot model")
            w[: v.numel()] = v.float()
        elif "nonZeroIndices" in params:
            idx = self._vec(params, "nonZeroIndices").long()
            val = self._vec(params, "nonZeroWeights", idx.numel()).float()
            if idx.numel() and (idx.min() < 0 or idx.max() >= self.dim - 1):
                raise ValueError(f"{self.NAME}: weight index out of range")
            w[idx] = val
        if self.rule.bias and params.get("intercept") is not None:
            w[self.dim - 1] = float(params["intercept"])
        self.w.copy_(w.to(self.device))
        self.on_state_loaded()

    def data_structure(self) -> dict:
        return {**super().data_structure(), "dim": self.dim, "numerical": self.space.dn,
                "nonZero": int((self.w != 0).sum()),
                "categorical": self.space.dc, "modelDtype": "bf16" if self.w16 is not None else "fp32"}


class PA(LinearLearner):
    NAME = "PA"


class SVM(LinearLearner):
    NAME = "SVM"


class RegressorPA(LinearLearner):
    NAME = "RegressorPA"
    TASK = "regression"
    RULE = L.RULE_EPS


class LogisticRegression(LinearLearner):
    NAME = "LogisticRegression"
    RULE = L.RULE_LOGISTIC
