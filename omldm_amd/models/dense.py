"""Dense-feature learners: ORR, K-means, NN (MLP) and HT (Hoeffding tree), plus the
hashed MultiClassPA.

Reference learner names: omldm/utils/parsers/requestStream/PipelineMap.scala:68; rules
[lit] in SURVEY.md Appendix D. Dense learners consume the dense block of the micro-batch
(numerical ∥ discrete features after the pipeline's preprocessors); hashed categorical
slots feed the linear family and MultiClassPA.
"""
from __future__ import annotations

import os

import math

import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.models.base import Learner, RoundContext, hp_float, hp_int
from omldm_amd.ops import dense as D
from omldm_amd.ops import linear as L


def _in_dim(h: dict, space: FeatureSpace) -> int:
    return int(h.get("_inDim", space.dn))


# ---------------------------------------------------------------------------- ORR

def _host_scalar(owner, v: float) -> torch.Tensor:
    """Device scalar holding ``v``, cached per value on ``owner`` (one H2D per distinct
    value, none per round): the active-spoke count the apply kernel divides by."""
    cache = owner.__dict__.setdefault("_scalar_cache", {})
    t = cache.get(v)
    if t is None:
        t = cache[v] = torch.full((1,), float(v), dtype=torch.float32, device=owner.device)
    return t

class ORR(Learner):
    """Online ridge regression: A = λI + Σxxᵀ, b = Σyx, w = A⁻¹b (intercept included).
    State = the augmented Gram matrix of [x, 1, y] — additive sufficient statistics, so
    worker merges are sums (merge_mode "sum") and exact. The per-round update is one
    MFMA pass (csrc/kernels/dense_learners.hip: gram_mfma_kernel) into an fp32 round
    buffer that starts at zero (bounded: one round's rows), folded into the fp64 master
    Gram — the reference keeps Breeze fp64 matrices, and an fp32 running sum of an
    unbounded stream stops absorbing rows. The solve is a Cholesky factorisation of the
    (d+1)×(d+1) system, refreshed lazily."""

    NAME = "ORR"
    TASK = "regression"
    merge_mode = "sum"
    supports_poly2_map = True  # fit() accepts an unexpanded PolyBatch (fused Gram kernel)

    def __init__(self, hyper, space, device="cpu"):
        super().__init__(hyper, space, device)
        self.d = _in_dim(self.hyper, space)
        self.ld = ((self.d + 2 + 31) // 32) * 32
        self.G = torch.zeros((self.ld, self.ld), dtype=torch.float64, device=self.device)
        self._G32 = torch.zeros((self.ld, self.ld), dtype=torch.float32, device=self.device)
        self._w = None
        self._retune()

    def fit(self, batch, ctx):
        if batch.B:
            self._G32.zero_()
            D.gram_update(batch.num.float(), batch.y, self._G32, cnt=self.cum[1:2],
                          pairs=getattr(batch, "pairs", None))
            self.G += self._G32
        self._w = None

    def state_vector(self):
        return self.G.view(-1)

    def on_state_loaded(self):
        self._w = None

    def weights(self) -> torch.Tensor:
        if self._w is None:
            d = self.d
            A = self.G[: d + 1, : d + 1].double()
            eye = torch.eye(d + 1, dtype=A.dtype, device=A.device)
            if self.lam > 0:
                A = A + self.lam * eye
            else:
                # λ = 0: a relative jitter keeps A positive definite, so the Cholesky solve
                # never has to be checked on the host (no device → host sync per predict)
                A = A + (1e-12 * (torch.diagonal(A).sum() / (d + 1)) + 1e-30) * eye
            b = self.G[: d + 1, d + 1].double()
            Lc, _ = torch.linalg.cholesky_ex(A)
            self._w = torch.cholesky_solve(b.unsqueeze(1), Lc).squeeze(1).float()
        return self._w

    def predict(self, batch):
        w = self.weights()
        return batch.num.float() @ w[: self.d] + w[self.d]

    def evaluate(self, batch):
        ok = ~torch.isnan(batch.y)
        e = (batch.y - self.predict(batch))[ok]
        se = (e * e).sum()
        return se, se, int(ok.sum())

    def _retune(self):
        lam = hp_float(self.hyper, "lambda", 1.0)
        if not lam >= 0:
            raise ValueError("ORR lambda must be >= 0")
        self.lam = lam
        self._w = None

    def parameters_map(self):
        d = self.d
        w = self.weights().cpu()
        return {"weights": w[:d].tolist(), "intercept": float(w[d]),
                "fitted": int(round(float(self.cum[1]))),
                # the sufficient statistics [x, 1, y]ᵀ[x, 1, y], row-major (d+2)²: what
                # a warm-started learner needs to keep learning exactly
                "gram": self.G[: d + 2, : d + 2].cpu().flatten().tolist()}

    def load_parameters(self, params):
        d = self.d
        G = torch.zeros((self.ld, self.ld), dtype=torch.float64)
        if params.get("gram") is not None:
            G[: d + 2, : d + 2] = self._vec(params, "gram", (d + 2) ** 2).view(d + 2, d + 2)
        else:  # weights only: b = λ·w with A = λI reproduces w (needs λ > 0)
            if not self.lam > 0:
                raise ValueError("ORR: importing weights without 'gram' needs lambda > 0")
            w = torch.cat([self._vec(params, "weights", d),
                           torch.tensor([float(params.get("intercept", 0.0))], dtype=torch.float64)])
            G[: d + 1, d + 1] = self.lam * w
            G[d + 1, : d + 1] = self.lam * w
        self.G.copy_(G.to(self.device))
        if params.get("fitted") is not None:
            self.cum[1] = float(params["fitted"])
        self._w = None

    def hyper_parameters(self):
        return {**super().hyper_parameters(), "lambda": self.lam}


# ------------------------------------------------------------------------- K-means
class KMeans(Learner):
    """Online k-means. Runs in SingleLearner mode (the reference forces it for K-means:
    omldm/operators/spoke/FlinkSpoke.scala:203-209).

    ``mode: "sequential"`` (the default, at any k and d ≤ 8192): the reference learner's
    exact per-point update — each training point, in stream order, moves its nearest
    centroid by c ← c + (x − c)/n_c; the first k points seed the centroids
    (csrc/kernels/kmeans_seq.hip: k ≤ 64 on one wavefront, G lanes per centroid; k ≤ 1024
    on four waves exchanging their minima through LDS; past the LDS the centroids stay in
    HBM). ``mode: "minibatch"``: assignments of a whole micro-batch against the batch-start
    centroids on the matrix cores, then c ← (n·c + Σx)/(n + m) (the same update summed over
    the batch; tests pin its quality gap against the sequential form)."""

    NAME = "K-means"
    TASK = "clustering"
    merge_mode = "mean"
    STRUCTURAL = ("k",)

    def structural_values(self):
        return {"k": self.k}

    def __init__(self, hyper, space, device="cpu"):
        super().__init__(hyper, space, device)
        self.k = hp_int(self.hyper, "k", 8)
        self.d = _in_dim(self.hyper, space)
        self.state = torch.zeros(self.k * self.d + self.k, dtype=torch.float32, device=self.device)
        self.C = self.state[: self.k * self.d].view(self.k, self.d)
        self.n = self.state[self.k * self.d:]
        self._sums = torch.zeros_like(self.C)
        self._cnt = torch.zeros_like(self.n)
        self._inert = torch.zeros(1, dtype=torch.float32, device=self.device)
        self._seeded = 0
        self._retune()

    def _retune(self) -> None:
        mode = str(self.hyper.get("mode", "sequential")).lower()
        self.sequential = mode != "minibatch" and D.kmeans_seq_fits(self.d, self.k)

    def fit(self, batch, ctx):
        if batch.B == 0:
            return
        if self.sequential:
            D.kmeans_seq(batch.num, batch.y, self.C, self.n, self.cum)
            return
        x = batch.num.float()
        if self._seeded < self.k:  # seed centroids with the first k training points
            train = ~torch.isnan(batch.y)
            rows = x[train][: self.k - self._seeded]
            m = rows.shape[0]
            self.C[self._seeded:self._seeded + m] = rows
            self.n[self._seeded:self._seeded + m] = 1.0
            self._seeded += m
        if self.device.type == "cuda":  # Σx/cnt are left at zero by the previous apply
            D.kmeans_assign(x, batch.y, self.C, self._sums, self._cnt, self._inert)
            D.kmeans_apply(self.C, self.n, self._sums, self._cnt, self._inert, self.cum)
            return
        self._sums.zero_()
        self._cnt.zero_()
        D.kmeans_assign(x, batch.y, self.C, self._sums, self._cnt, self._inert)
        tot = self.n + self._cnt
        upd = tot > 0
        newc = (self.C * self.n.unsqueeze(1) + self._sums) / torch.clamp(tot, min=1).unsqueeze(1)
        self.C.copy_(torch.where(upd.unsqueeze(1), newc, self.C))
        self.n.copy_(tot)
        self.cum[1] += (~torch.isnan(batch.y)).sum()
        self.cum[0] += self._inert[0]
        self._inert.zero_()

    def state_vector(self):
        return self.state

    def predict(self, batch):
        a = D.kmeans_assign(batch.num.float(), None, self.C, None, None, want_assign=True)
        return a.float()

    def evaluate(self, batch):
        x = batch.num.float()
        dist = torch.cdist(x, self.C) ** 2
        inert = dist.min(1).values.sum()
        return inert, inert, batch.B

    def parameters_map(self):
        return {"centroids": self.C.cpu().flatten().tolist(), "counts": self.n.cpu().tolist(),
                "k": self.k, "dim": self.d}

    def load_parameters(self, params):
        C = self._vec(params, "centroids", self.k * self.d).float().view(self.k, self.d)
        n = self._vec(params, "counts", self.k).float()
        self.C.copy_(C.to(self.device))
        self.n.copy_(n.to(self.device))
        self._seeded = self.k  # imported centroids count as seeded
        if self.sequential:  # the sequential kernel reads seeding from n > 0
            self.n.clamp_(min=1.0)


# ---------------------------------------------------------------------- MultiClassPA
class MultiClassPA(Learner):
    """K-prototype Passive-Aggressive classifier on hashed features (labels 0..K-1);
    virtual spokes per round: on a GPU with the field-aware wire and K ≤ 16 the v3 table scan
    (csrc/kernels/linear_scan3.hip: s3mc_scan_kernel), else the spoke tables
    (csrc/kernels/multiclass_spoke.hip)."""

    NAME = "MultiClassPA"
    TASK = "classification"
    merge_mode = "mean"
    STRUCTURAL = ("nClasses",)

    def structural_values(self):
        return {"nClasses": self.K}

    def _retune(self) -> None:
        v = str(self.hyper.get("variant", "PA-I"))
        C = hp_float(self.hyper, "C", 1.0)
        if not C > 0:
            raise ValueError("MultiClassPA C must be > 0")
        self.variant = {"PA": 0, "PA-I": 1, "PA-II": 2}.get(v, 1)
        self.C = C
        self.bias = bool(self.hyper.get("bias", True))

    def __init__(self, hyper, space, device="cpu"):
        super().__init__(hyper, space, device)
        self.K = max(2, hp_int(self.hyper, "nClasses", 2))
        self.dim = space.dim
        self.W = torch.zeros((self.K, self.dim), dtype=torch.float32, device=self.device)
        self.dacc = torch.zeros_like(self.W)
        self.st = torch.zeros(8, dtype=torch.float32, device=self.device)
        self._retune()
        # GPU: key-major prototype shadow for the round's gathers (fp32, or bf16 with
        # modelDtype=bf16), refreshed by the apply pass and on every state load
        self.Wt = None
        if self.device.type == "cuda":
            bf16 = str(self.hyper.get("modelDtype", "fp32")).lower() in ("bf16", "bfloat16")
            self.Wt = D.proto_shadow(self.W, torch.bfloat16 if bf16 else torch.float32)

    def on_state_loaded(self):
        if self.Wt is not None:
            self.Wt[:, : self.K].copy_(self.W.t())

    def _fit_two_classes(self, batch, ctx, R: int, S: int) -> bool:
        """Two classes are one binary PA on v = w_0 − w_1: with y' = +1 for class 0 and −1
        for class 1, the margin s_y − s_r is y'·v·x, the hinge loss is the same, the update
        moves w_y by +τx and w_r by −τx, i.e. v by y'·2τ·x, and w_0 + w_1 never changes;
        2τ is the binary step at C' = 2C (PA-I: min(2C, ℓ/‖x‖²); PA-II: ℓ/(‖x‖² + 1/(4C));
        PA: ℓ/‖x‖²). So the round runs the binary v3 scan (its step chain is ~4× shorter
        than the K-score scan's) and the prototypes are rebuilt from v and the invariant
        sum. Same rows, same order, same running totals (hinge loss, margin ≤ 0 mistakes)."""
        from omldm_amd.api.batch import RawBatch

        if not (self.W.is_cuda and os.environ.get("OMLDM_MC_BINARY", "1") != "0"
                and self.Wt is not None and self.Wt.dtype == torch.float32
                and getattr(batch, "cat_span", 0) > 0 and batch.dc > 0 and batch.y.is_cuda
                and L.SEQ_KERNEL == "scan3"
                and batch.dn + batch.dc * batch.cat_span <= self.dim - 1
                and L.scan3_fits(batch.dn, batch.dc, R, self.bias)):
            return False
        yf = batch.y.float()
        yb = torch.where(yf == 0, 1.0, torch.where(yf == 1, -1.0, float("nan"))).contiguous()
        rb = RawBatch(batch.num.float().contiguous(), batch.cat.contiguous(), yb,
                      span=batch.cat_span, cbase=batch.dn)
        if not L.scan3_eligible_compact(rb, R, self.bias, self.dim):
            return False
        rule = L.LinearRule(rule=L.RULE_HINGE, variant=self.variant, C=2.0 * self.C,
                            bias=self.bias)
        if getattr(self, "_dacc2", None) is None:
            self._dacc2 = torch.zeros(self.dim + 2, dtype=torch.float32, device=self.device)
        ssum = self.W[0] + self.W[1]
        v = (self.W[0] - self.W[1]).contiguous()
        L.linear_seq_round(v, rb, R, S, self._dacc2, rule, ctx.inv_p, cum=self.cum,
                           hashed=True)
        L.linear_apply(v, None, self._dacc2)
        self.W[0].copy_((ssum + v) * 0.5)
        self.W[1].copy_((ssum - v) * 0.5)
        self.on_state_loaded()  # the key-major shadow
        return True

    def fit(self, batch, ctx):
        if batch.B == 0:
            return
        S = max(1, ctx.spokes)
        R = max(1, -(-batch.B // S))
        if self.K == 2 and self._fit_two_classes(batch, ctx, R, S):
            return
        if D.multiclass_scan3_fits(batch, R, self.K, self.bias, self.Wt):
            # exact sequential spokes on the v3 table scan (K ≤ 16, field-aware wire)
            D.multiclass_scan3_round(self.Wt, batch, R, S, self.K, self.variant, self.C,
                                     self.bias, self.dacc, self.st)
        else:  # the spoke-table round (LDS delta tables spilling to HBM)
            D.multiclass_round(self.W, batch, R, S, self.K, self.variant, self.C, self.bias,
                               self.dacc, self.st, log2cap=hp_int(self.hyper, "tableLog2", 0),
                               Wt=self.Wt)
        # every spoke with rows is active: ceil(B / R) of them, known on the host
        D.multiclass_apply(self.W, self.dacc, _host_scalar(self, -(-batch.B // R)), self.Wt,
                           st=self.st, cum=self.cum, fold=1)

    def state_vector(self):
        return self.W.view(-1)

    def scores(self, batch):
        return L.linear_predict(self.W, batch.to_wide(), bias=self.bias)

    def predict(self, batch):
        return self.scores(batch).argmax(1).float()

    def evaluate(self, batch):
        ok = ~torch.isnan(batch.y)
        if batch.B == 0 or not bool(ok.any()):
            z = torch.zeros((), device=self.device)
            return z, z, 0
        s = self.scores(batch)[ok]
        y = batch.y[ok].long().clamp(0, self.K - 1)
        sy = s.gather(1, y.unsqueeze(1)).squeeze(1)
        s2 = s.clone()
        s2.scatter_(1, y.unsqueeze(1), float("-inf"))
        loss = torch.clamp(1 - (sy - s2.max(1).values), min=0).sum()
        return loss, (s.argmax(1) == y).float().sum(), int(ok.sum())

    def parameters_map(self):
        """K prototypes over the hashed feature space, row-major [K, dim] (intercept in the
        last slot of each row)."""
        return {"weights": self.W.detach().float().cpu().flatten().tolist(),
                "nClasses": self.K, "dim": self.dim}

    def load_parameters(self, params):
        if params.get("weights") is not None:
            W = self._vec(params, "weights", self.K * self.dim).float().view(self.K, self.dim)
        else:
            W = torch.zeros((self.K, self.dim), dtype=torch.float32)
            idx = self._vec(params, "nonZeroIndices").long()
            W.view(-1)[idx] = self._vec(params, "nonZeroWeights", idx.numel()).float()
        self.W.copy_(W.to(self.device))
        self.on_state_loaded()


# ------------------------------------------------------------------------------ NN
class NN(Learner):
    """Multi-layer perceptron (ReLU / tanh / sigmoid / identity hidden layers,
    ``activation`` hyper-parameter) trained by mini-batch SGD — the
    reference's DL4J MultiLayerNetwork path (hs_err_pid77107.log:97-110).

    A round runs S virtual spokes (one workgroup each, csrc/kernels/mlp.hip): spoke s does
    32-row mini-batch SGD over its rows from the round-start model entirely in LDS on the
    fp32 matrix cores; the spokes' models are then averaged (intra-GPU hub). Parameters
    live in ONE flat fp32 buffer (W_0, b_0, W_1, b_1, … row-major) — the protocols' state
    vector. Loss: squared error (task=regression), logistic (nClasses ≤ 1, labels ±1 or
    {0,1}) or softmax cross-entropy (nClasses = K ≥ 2). At most 4 layers whose padded
    widths fit the 160 KB LDS of a CU (e.g. 128-wide hidden layers)."""

    NAME = "NN"
    merge_mode = "mean"
    MB = D.MLP_MB
    STRUCTURAL = ("hiddenLayers", "nClasses", "task", "seed")

    def structural_values(self):
        return {"hiddenLayers": list(self.widths[1:-1]), "nClasses": self.K,
                "task": self.TASK, "seed": self.seed}

    def _retune(self) -> None:  # learning rate, activation and matmul precision
        h = self.hyper
        act = str(h.get("activation", "relu")).lower()
        if act not in D.MLP_ACTS:
            raise ValueError(f"NN activation must be one of {sorted(D.MLP_ACTS)}")
        self.lr = hp_float(h, "learningRate", 0.05)
        self.act_name, self.act = act, D.MLP_ACTS[act]
        if str(h.get("matmulDtype", "fp32")).lower() in ("bf16", "bfloat16"):
            self.act |= D.MLP_BF16

    def __init__(self, hyper, space, device="cpu"):
        super().__init__(hyper, space, device)
        h = self.hyper
        self.d = _in_dim(h, space)
        hidden = h.get("hiddenLayers", [32, 32])
        if isinstance(hidden, str):
            hidden = [int(v) for v in hidden.strip("[]").split(",") if v.strip()]
        self.K = hp_int(h, "nClasses", 1)   # 1: binary (±1 or {0,1}) / regression output
        self.TASK = "regression" if str(h.get("task", "classification")) == "regression" \
            else "classification"
        self.task_id = 0 if self.TASK == "regression" else (1 if self.K <= 1 else 2)
        self.lr = hp_float(h, "learningRate", 0.05)
        act = str(h.get("activation", "relu")).lower()
        if act not in D.MLP_ACTS:
            raise ValueError(f"NN activation must be one of {sorted(D.MLP_ACTS)}")
        self.act_name, self.act = act, D.MLP_ACTS[act]
        # matmulDtype bf16: GEMM operands rounded to bf16 on the matrix cores (fp32
        # accumulation, fp32 master weights and activations in LDS) — K/16 MFMAs per tile
        # instead of K/2; default fp32 keeps DL4J's fp32 arithmetic
        if str(h.get("matmulDtype", "fp32")).lower() in ("bf16", "bfloat16"):
            self.act |= D.MLP_BF16
        self.seed = hp_int(h, "seed", hp_int(h, "_seed", 25))
        self.widths = [self.d] + [int(v) for v in hidden] + [max(1, self.K)]
        if len(self.widths) - 1 > D.MLP_MAX_LAYERS:
            raise ValueError(f"NN supports at most {D.MLP_MAX_LAYERS} layers")
        self.shapes = []
        for a, b in zip(self.widths[:-1], self.widths[1:]):
            self.shapes += [(b, a), (b,)]
        total = sum(math.prod(s) for s in self.shapes)
        g = torch.Generator().manual_seed(self.seed)
        flat = torch.zeros(total, dtype=torch.float32)
        o = 0
        for s in self.shapes:
            n = math.prod(s)
            if len(s) == 2:
                flat[o:o + n] = torch.randn(n, generator=g) * math.sqrt(2.0 / s[1])
            o += n
        self.flat = flat.to(self.device)
        self.dacc = torch.zeros_like(self.flat)
        self.st = torch.zeros(8, dtype=torch.float32, device=self.device)
        self._nact = torch.zeros(2, dtype=torch.float32, device=self.device)
        self._parity = 0
        if self.device.type == "cuda" and D.mlp_lds_bytes(self.widths) > 160 * 1024:
            raise ValueError("NN layer widths exceed the LDS budget of the fused kernel")

    def fit(self, batch, ctx):
        B = batch.B
        if B == 0:
            return
        S = max(1, ctx.spokes)
        per = -(-B // S)
        R = -(-per // self.MB) * self.MB
        S = -(-B // R)
        # divisor = spokes with ≥ 1 labelled row, counted by the round kernel on the device
        # (rows with NaN targets make no update); two buffers alternate so the apply can
        # zero the next round's while it reads this round's
        k = self._parity
        self._parity ^= 1
        D.mlp_round(self.flat, batch.num, batch.y, R, S, self.widths, self.task_id, self.lr,
                    self.dacc, self.st, self.act, nact=self._nact[k:k + 1])
        D.multiclass_apply(self.flat, self.dacc, self._nact[k:k + 1], st=self.st,
                           cum=self.cum, fold=3 if self.task_id else 2,
                           nact_next=self._nact[k ^ 1:(k ^ 1) + 1])

    def state_vector(self):
        return self.flat

    def forward(self, x):
        return D.mlp_forward(self.flat, x.float(), self.widths, self.act)

    def predict(self, batch):
        out = self.forward(batch.num)
        if self.task_id == 0:
            return out[:, 0]
        if self.task_id == 1:
            return torch.where(out[:, 0] >= 0, 1.0, -1.0)
        return out.argmax(1).float()

    def evaluate(self, batch):
        ok = ~torch.isnan(batch.y)
        if not bool(ok.any()):
            z = torch.zeros((), device=self.device)
            return z, z, 0
        out = self.forward(batch.num)[ok]
        y = batch.y[ok]
        _, loss, correct = D._mlp_grad_out(out, y, self.task_id, max(1, self.K))
        score = loss if self.task_id == 0 else correct
        return loss, score, int(ok.sum())

    def hyper_parameters(self):
        return {**super().hyper_parameters(), "learningRate": self.lr, "miniBatchSize": self.MB,
                "activation": self.act_name}

    def parameters_map(self):
        """Per layer l: ``W{l}`` (out × in, row-major) and ``b{l}`` — DL4J's
        MultiLayerNetwork parameter table, flattened."""
        out = {"layers": [list(s) for s in self.shapes[::2]]}
        flat = self.flat.detach().float().cpu()
        o = 0
        for i, s in enumerate(self.shapes):
            n = math.prod(s)
            out[("W" if len(s) == 2 else "b") + str(i // 2)] = flat[o:o + n].tolist()
            o += n
        return out

    def load_parameters(self, params):
        flat = torch.empty(self.flat.numel(), dtype=torch.float32)
        o = 0
        for i, s in enumerate(self.shapes):
            n = math.prod(s)
            flat[o:o + n] = self._vec(params, ("W" if len(s) == 2 else "b") + str(i // 2), n).float()
            o += n
        self.flat.copy_(flat.to(self.device))


# ------------------------------------------------------------------------------ HT
class HT(Learner):
    """Hoeffding tree (VFDT) for classification on dense features.

    Leaves keep class counts and per-(feature, class) Gaussian sufficient statistics
    (n, Σx, Σx²); every ``gracePeriod`` points a leaf evaluates ``nBins`` candidate
    thresholds per feature (class mass split by the Gaussian CDFs), and splits when the
    information-gain lead of the best attribute beats the Hoeffding bound
    ε = sqrt(R² ln(1/δ) / (2n)) or ε < τ (tie). Routing, statistics and split search
    are batched tensor ops on the device; the tree is flat arrays (state vector)."""

    NAME = "HT"
    merge_mode = "mean"
    STRUCTURAL = ("nClasses", "maxNodes", "maxDepth", "nBins")

    def structural_values(self):
        return {"nClasses": self.Cn, "maxNodes": self.N, "maxDepth": self.depth,
                "nBins": self.nb}

    def _retune(self) -> None:
        self.grace = hp_int(self.hyper, "gracePeriod", 200)
        self.delta = hp_float(self.hyper, "delta", 1e-7)
        self.tau = hp_float(self.hyper, "tau", 0.05)
        # checkEvery 0 (default): a leaf is checked at the very point it reaches the grace
        # period, as the reference's per-point VFDT (the tick is cut into segments ending at
        # each due point: _fit_exact). checkEvery N > 0: due leaves are checked every N rows
        # (faster; tests/test_ht_sequential.py pins its gap to the per-point form)
        self.check_every = max(0, hp_int(self.hyper, "checkEvery", 0))
        # exactDevice (default true): the exact mode's tick runs in one persistent launch;
        # false keeps the host-driven segment loop (the A/B reference of the same semantics)
        self.exact_device = str(self.hyper.get("exactDevice", True)).lower() not in ("0", "false")

    def __init__(self, hyper, space, device="cpu"):
        super().__init__(hyper, space, device)
        h = self.hyper
        self.d = _in_dim(h, space)
        self.Cn = max(2, hp_int(h, "nClasses", 2))
        self.N = hp_int(h, "maxNodes", 255)
        self.depth = hp_int(h, "maxDepth", 12)
        self.grace = hp_int(h, "gracePeriod", 200)
        self.delta = hp_float(h, "delta", 1e-7)
        self.tau = hp_float(h, "tau", 0.05)
        self.nb = hp_int(h, "nBins", 16)
        self._retune()
        dev = self.device
        N, d, C = self.N, self.d, self.Cn
        # flat state: feature, threshold, left, right, class counts, S0, S1, S2, lo, hi, since
        self.sizes = [N, N, N, N, N * C, N * d * C, N * d * C, N * d * C, N * d, N * d, N, 1]
        self.state = torch.zeros(sum(self.sizes), dtype=torch.float32, device=dev)
        v = torch.split(self.state, self.sizes)
        self.feat, self.thr, self.left, self.right = v[0], v[1], v[2], v[3]
        self.cc = v[4].view(N, C)
        self.S0, self.S1, self.S2 = (t.view(N, d, C) for t in v[5:8])
        self.lo, self.hi = v[8].view(N, d), v[9].view(N, d)
        self.since = v[10]
        self.nnodes = v[11]
        self.feat.fill_(-1)
        self.lo.fill_(float("inf"))
        self.hi.fill_(float("-inf"))
        self.nnodes.fill_(1)

    def _route(self, x):
        node = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
        for _ in range(self.depth + 1):
            f = self.feat[node].long()
            inner = f >= 0
            if not bool(inner.any()):
                break
            xv = x.gather(1, f.clamp(min=0).unsqueeze(1)).squeeze(1)
            go_left = xv <= self.thr[node]
            nxt = torch.where(go_left, self.left[node], self.right[node]).long()
            node = torch.where(inner, nxt, node)
        return node

    def _tree(self):
        return [self.feat, self.thr, self.left, self.right, self.cc, self.S0, self.S1, self.S2,
                self.lo, self.hi, self.since, self.nnodes]

    def fit(self, batch, ctx):
        B, step = batch.B, self.check_every
        if step <= 0:
            return self._fit_exact(batch)
        if B > step:
            for a in range(0, B, step):
                self._fit_part(batch.slice(a, min(B, a + step)))
            return
        self._fit_part(batch)

    def _fit_exact(self, batch):
        """Per-point VFDT checks: the tick is cut into segments that end exactly at the next
        row where some leaf reaches its grace period (rows of each leaf in stream order: the
        (grace − since)-th training row of the leaf); each segment's statistics are added,
        then the due leaf is checked; rows after a split are routed again. GPU: the whole
        loop is one persistent launch (D.ht_exact); the host-driven form below (one launch
        per segment) is the CPU path and the A/B reference (exactDevice false)."""
        import numpy as np

        B = batch.B
        if B == 0:
            return
        gpu = self.device.type == "cuda"
        x = batch.num.float().contiguous()
        if gpu and self.exact_device and D.ht_exact(
                x, batch.y, self.Cn, self.depth, self.N, self.nb, float(self.grace), self.delta,
                self.tau, self._tree(), self.cum[1:2]):
            return  # one persistent launch for the tick (csrc/kernels/hoeffding.hip)
        ok = (~torch.isnan(batch.y)).cpu().numpy()
        N, g = self.N, float(self.grace)

        def route(xs):
            if gpu:
                return D.ht_route(xs, self.depth, self._tree()).cpu().numpy().astype(np.int64)
            return self._route(xs).cpu().numpy().astype(np.int64)

        def update(lo, hi, check):  # rows [lo, hi): statistics, then the due leaves' checks
            if not gpu:  # (the CPU path checks inside _fit_part)
                self._fit_part(batch.slice(lo, hi))
                return
            # (the sorted reducer even for short segments: the atomic form serialises on the
            # few leaves a segment's rows share — 5x slower per check, profiles/round5)
            D.ht_update(x[lo:hi], batch.y[lo:hi], self.Cn, self.depth, self._tree(),
                        self.cum[1:2], N=self.N)
            if check:
                D.ht_split(self.N, self.d, self.Cn, self.nb, g, self.delta, self.tau,
                           self._tree())

        a = 0
        while a < B:
            leaf = route(x[a:])
            since = self.since.cpu().numpy().astype(np.float64)
            isleaf = (self.feat.cpu().numpy() < 0)
            nodes0 = int(self.nnodes.item())
            rel = np.flatnonzero(ok[a:])                  # training rows, relative to a
            lv = leaf[rel]
            # by leaf, then stream position (rel ascends: a stable radix sort on the leaf)
            order = np.argsort(lv.astype(np.uint8 if N <= 256 else np.uint16), kind="stable")
            lv_s, pos_s = lv[order], rel[order]
            cnt = np.bincount(lv_s, minlength=N)[:N]
            start = np.concatenate([[0], np.cumsum(cnt)[:-1]])
            keys = lv_s * (B + 1) + pos_s
            done = np.zeros(N, dtype=np.int64)             # rows of each leaf consumed
            e = 0                                          # rows [a, a + e) processed
            split = False
            while e < B - a:
                need = np.maximum(1, np.ceil(g - since)).astype(np.int64)
                idx = start + done + need - 1
                due = (done + need <= cnt) & isleaf
                if not due.any():
                    break
                first = int(pos_s[idx[due]].min())         # the earliest due row
                end = first + 1
                update(a + e, a + end, True)
                newdone = np.searchsorted(keys, np.arange(N) * (B + 1) + end) - start
                since += newdone - done
                done = newdone
                since[since >= g] = 0.0                    # the checked leaf (ht_split)
                e = end
                if int(self.nnodes.item()) != nodes0:      # a split: route the rest again
                    split = True
                    break
            if not split:
                if e < B - a:  # no leaf reaches its grace period in the rest of the tick
                    update(a + e, B, False)
                return
            a += e

    def _fit_part(self, batch):
        if self.device.type == "cuda":
            # device path (csrc/kernels/hoeffding.hip): no host synchronisation per round
            if batch.B:
                D.ht_update(batch.num, batch.y, self.Cn, self.depth, self._tree(),
                            self.cum[1:2], N=self.N)
                D.ht_split(self.N, self.d, self.Cn, self.nb, float(self.grace), self.delta,
                           self.tau, self._tree())
            return
        ok = ~torch.isnan(batch.y)
        if not bool(ok.any()):
            return
        x = batch.num.float()[ok]
        y = batch.y[ok].long().clamp(0, self.Cn - 1)
        y = torch.where(y < 0, 0, y)
        leaf = self._route(x)
        N, d, C = self.N, self.d, self.Cn
        self.cc.view(-1).index_add_(0, leaf * C + y, torch.ones_like(y, dtype=torch.float32))
        idx = ((leaf * d).unsqueeze(1) + torch.arange(d, device=x.device)) * C + y.unsqueeze(1)
        self.S0.view(-1).index_add_(0, idx.reshape(-1), torch.ones(idx.numel(), device=x.device))
        self.S1.view(-1).index_add_(0, idx.reshape(-1), x.reshape(-1))
        self.S2.view(-1).index_add_(0, idx.reshape(-1), (x * x).reshape(-1))
        li = (leaf * d).unsqueeze(1) + torch.arange(d, device=x.device)
        self.lo.view(-1).scatter_reduce_(0, li.reshape(-1), x.reshape(-1), "amin")
        self.hi.view(-1).scatter_reduce_(0, li.reshape(-1), x.reshape(-1), "amax")
        self.since.index_add_(0, leaf, torch.ones(leaf.shape[0], device=x.device))
        self.cum[1] += x.shape[0]
        self._try_split()

    @staticmethod
    def _entropy(counts):
        tot = counts.sum(-1, keepdim=True).clamp(min=1e-12)
        p = counts / tot
        return -(p * torch.log2(p.clamp(min=1e-12))).sum(-1)

    def _try_split(self):
        cand = torch.nonzero((self.since >= self.grace) & (self.feat < 0)).flatten()
        if cand.numel() == 0:
            return
        for node in cand.tolist():
            n_total = float(self.cc[node].sum())
            self.since[node] = 0
            if n_total < 2 or int(self.nnodes.item()) + 2 > self.N:
                continue
            cc = self.cc[node]
            if int((cc > 0).sum()) < 2:
                continue
            S0, S1, S2 = self.S0[node], self.S1[node], self.S2[node]  # [d, C]
            mu = S1 / S0.clamp(min=1)
            var = (S2 / S0.clamp(min=1) - mu * mu).clamp(min=1e-6)
            sd = var.sqrt()
            lo, hi = self.lo[node], self.hi[node]
            span = (hi - lo).clamp(min=0)
            q = torch.linspace(0, 1, self.nb + 2, device=S0.device)[1:-1]
            t = lo.unsqueeze(1) + span.unsqueeze(1) * q.unsqueeze(0)      # [d, nb]
            z = (t.unsqueeze(2) - mu.unsqueeze(1)) / sd.unsqueeze(1)      # [d, nb, C]
            cdf = 0.5 * (1 + torch.erf(z / math.sqrt(2)))
            left = S0.unsqueeze(1) * cdf                                  # [d, nb, C]
            right = S0.unsqueeze(1) - left
            nl, nr = left.sum(-1), right.sum(-1)
            h0 = self._entropy(cc)
            gain = h0 - (nl * self._entropy(left) + nr * self._entropy(right)) / \
                (nl + nr).clamp(min=1e-12)
            gain = torch.where(span.unsqueeze(1) > 0, gain, torch.full_like(gain, -1))
            per_feat, arg = gain.max(1)
            order = torch.argsort(per_feat, descending=True)
            g1 = float(per_feat[order[0]])
            g2 = float(per_feat[order[1]]) if self.d > 1 else 0.0
            R = math.log2(self.Cn)
            eps = math.sqrt(R * R * math.log(1.0 / self.delta) / (2.0 * n_total))
            if g1 > 0 and (g1 - g2 > eps or eps < self.tau):
                f = int(order[0])
                thr = float(t[f, arg[f]])
                nn = int(self.nnodes.item())
                lch, rch = nn, nn + 1
                self.nnodes += 2
                self.feat[node] = f
                self.thr[node] = thr
                self.left[node], self.right[node] = lch, rch
                # children start with the class mass estimated on each side
                self.cc[lch] = left[f, arg[f]]
                self.cc[rch] = right[f, arg[f]]

    def state_vector(self):
        return self.state

    def predict(self, batch):
        if self.device.type == "cuda":
            return D.ht_predict(batch.num, self.Cn, self.depth, self._tree())
        leaf = self._route(batch.num.float())
        return self.cc[leaf].argmax(1).float()

    def evaluate(self, batch):
        ok = ~torch.isnan(batch.y)
        if not bool(ok.any()):
            z = torch.zeros((), device=self.device)
            return z, z, 0
        p = self.predict(batch)[ok]
        y = batch.y[ok]
        err = (p != y).float().sum()
        return err, (p == y).float().sum(), int(ok.sum())

    _HT_ARRAYS = ("feature", "threshold", "left", "right", "classCounts", "S0", "S1", "S2",
                  "lo", "hi", "since")

    def parameters_map(self):
        """The tree (split feature / threshold / children / leaf class counts) and the
        leaves' sufficient statistics (Gaussian per-(feature, class) moments, ranges,
        points since the last split check), node-major over the ``nodes`` in use."""
        n = int(self.nnodes.item())
        arrs = self._tree()[:11]
        out = {"nodes": n}
        for name, t in zip(self._HT_ARRAYS, arrs):
            v = t[:n].detach().float().cpu().flatten()
            out[name] = [int(x) for x in v.tolist()] if name in ("feature", "left", "right") \
                else v.tolist()
        return out

    def load_parameters(self, params):
        n = int(params["nodes"])
        if not 1 <= n <= self.N:
            raise ValueError(f"HT: {n} nodes for a {self.N}-node tree")
        self.state.zero_()
        self.feat.fill_(-1)
        self.lo.fill_(float("inf"))
        self.hi.fill_(float("-inf"))
        for name, t in zip(self._HT_ARRAYS, self._tree()[:11]):
            per = t[0].numel() if t.dim() > 1 else 1
            v = self._vec(params, name, n * per).float().view((n,) + tuple(t.shape[1:]))
            t[:n].copy_(v.to(self.device))
        self.nnodes.fill_(n)
