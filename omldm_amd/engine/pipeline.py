"""One ML pipeline (= one reference ``networkId``): preprocessors → learner, driven by a
synchronisation protocol, plus its statistics.

Reference: a pipeline is created by a Create request (FlinkSpoke.createWrapper,
omldm/operators/spoke/FlinkSpoke.scala:177-224): parallel jobs force SingleLearner for
HT / K-means (:203-209), a single-worker job forces CentralizedTraining (:213-215), and
the protocol/hub parallelism come from ``trainingConfiguration`` (:181-190; factory
omldm/utils/generators/MLNodeGenerator.scala:20-76). Points are piped through the
preprocessors into the learner (MLPipeline.pipePoint, hs_err_pid77107.log:111).
"""
from __future__ import annotations

import collections

import os

import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch, PolyBatch
from omldm_amd.api.schemas import SINGLE_LEARNER_MODELS, Request
from omldm_amd.engine.statistics import merge_bucketed
from omldm_amd.models import make_learner, make_preprocessor
from omldm_amd.parallel.comm import Comm
from omldm_amd.parallel.protocols import make_protocol


class Pipeline:
    def __init__(self, request: Request, space: FeatureSpace, comm: Comm, device,
                 spokes: int, parallelism: int, max_msg_params: int = 10000, store=None,
                 seed: int = 25):
        self.id = int(request.id)
        self.request = request
        self.space = space
        self.device = device
        cfg = dict(request.trainingConfiguration or {})
        name = request.learner.name
        # Preprocessors first: they fix the learner's dense input width.
        self.preprocessors = [make_preprocessor(p.name, p.hyperParameters, device)
                              for p in (request.preProcessors or [])]
        d = space.dn
        for p in self.preprocessors:
            d = p.out_dim(d)
        hyper = dict(request.learner.hyperParameters or {})
        hyper["_inDim"] = d
        hyper["_seed"] = int(seed)  # the job's seed (Random.setSeed, FlinkSpoke.scala:52)
        # A widened dense block (PolynomialFeatures) keeps slots [0, d) for the hashed
        # learners; its top overlaps the lowest hashed slots like any hash collision.
        if d + 1 >= space.dim:
            raise ValueError("dense block wider than the hashed feature space")
        self.learner = make_learner(name, hyper, space, device)
        # warm start: a Create carrying the reference's portable model format — a
        # QueryResponse's learner.parameters / preprocessor parameters, bucketed keys
        # ``name[start-end]`` merged back (FlinkSpoke.scala:198-219 hands the request's
        # learner POJO to node creation)
        if request.learner.parameters:
            self.learner.load_parameters(merge_bucketed(request.learner.parameters))
        for pre, pojo in zip(self.preprocessors, request.preProcessors or []):
            if pojo.parameters:
                pre.load_parameters(merge_bucketed(pojo.parameters))
        # hashed-linear pipelines without preprocessors keep their weights in the shared
        # HBM model store so forecasts are scored for all of them in one launch
        self.store, self.store_row = None, None
        if store is not None and not self.preprocessors and hasattr(self.learner, "attach"):
            self.store = store
            self.store_row = store.add(self.learner)
        # Protocol selection rules of the reference.
        if parallelism <= 1 and comm.world == 1:
            proto = "CentralizedTraining"
        elif name in SINGLE_LEARNER_MODELS and comm.world > 1:
            proto = "SingleLearner"
        else:
            proto = cfg.get("protocol")
        if name in SINGLE_LEARNER_MODELS and comm.world == 1 and proto != "CentralizedTraining":
            cfg.setdefault("virtualSpokes", 1)
        cfg["_tag"] = self.id  # point-to-point message tag of this pipeline's PS channels
        self.protocol = make_protocol(proto, comm, self.learner, cfg, spokes=spokes,
                                      max_msg_params=max_msg_params)
        self.protocol_name = self.protocol.NAME
        # PolynomialFeatures(2) in front of a learner that fuses the map into its update
        # (ORR): training batches reach the learner unexpanded (api/batch.py: PolyBatch)
        last = self.preprocessors[-1] if self.preprocessors else None
        self._fuse_poly2 = (os.environ.get("OMLDM_FUSE_POLY", "1") != "0"  # A/B knob
                            and getattr(self.learner, "supports_poly2_map", False)
                            and last is not None and last.NAME == "PolynomialFeatures"
                            and last.degree == 2)
        # running statistics (reference Statistics / learning curve, FlinkHub.scala:95-156)
        self.learning_curve: list[tuple[float, int]] = []
        self._lc_last = (0.0, 0)
        # GPU: pinned copies of the running totals behind each tick's round, with their
        # events; a point is taken once its copy has landed (never waiting on the GPU while
        # fewer than LC_LAG ticks are in flight)
        self._lc_free: list = []
        self._lc_pending: collections.deque = collections.deque()
        # mean buffer size (reference BufferingWrapper.getMeanBufferSize): the training
        # records a spoke holds when its round starts — rows of the round / local spokes
        self.spokes = max(1, int(spokes))
        self._buf_sum, self._buf_rounds = 0.0, 0

    # --------------------------------------------------------------- data path
    def _pre(self, batch: HashedBatch, train: bool) -> HashedBatch:
        if train and self._fuse_poly2:
            for p in self.preprocessors[:-1]:
                batch = p(batch, train=True)
            pairs = self.preprocessors[-1].pair_index(batch.dn, batch.num.device)
            return PolyBatch(batch.num.float().contiguous(), batch.cat, batch.y, batch.raw,
                             batch.cat_span, pairs)
        for p in self.preprocessors:
            batch = p(batch, train=train)
        return batch

    def _note_buffer(self, rows: int) -> None:
        self._buf_sum += rows / self.spokes
        self._buf_rounds += 1

    def mean_buffer_size(self) -> float:
        return self._buf_sum / self._buf_rounds if self._buf_rounds else 0.0

    def train(self, batch: HashedBatch) -> None:
        """One protocol round on this rank's training rows (possibly empty)."""
        self._note_buffer(batch.B)
        self.protocol.round(self._pre(batch, True))

    def train_local(self, batch: HashedBatch) -> torch.Tensor:
        """Phase 1 of a split Synchronous round: train, return the buffer to reduce."""
        self._note_buffer(batch.B)
        return self.protocol.local(self._pre(batch, True))

    def predict(self, batch: HashedBatch) -> torch.Tensor:
        return self.learner.predict(self._pre(batch, False))

    def evaluate(self, batch: HashedBatch):
        return self.learner.evaluate(self._pre(batch, False))

    def close(self) -> None:
        # drain point-to-point channels (every rank deletes at the same tick), so a
        # pipeline re-created under the same id starts on clean channels
        self.protocol.finalize()
        if self.store is not None:
            self.store.remove(self.store_row)
            self.store = None

    def scores_to_predictions(self, s: torch.Tensor) -> torch.Tensor:
        """Decision values from the model store → this learner's prediction values."""
        if self.learner.TASK == "classification":
            return torch.where(s >= 0, 1.0, -1.0)
        return s

    # ticks whose curve copies may be in flight: 1 (take the previous tick's point) measured
    # best end to end — letting the host run further ahead put the next tick's round beside
    # its parse on the GPU (JSON e2e 60-64 → 53 M records/s, DIB no better), A/B:
    # OMLDM_LC_LAG (gpurun_out/r5/e2e_OMLDM_LC_LAG_*.json)
    LC_LAG = int(os.environ.get("OMLDM_LC_LAG", "1"))

    def record_learning_curve(self) -> None:
        """One learning-curve point per tick: (mean loss of the rows fitted since the last
        point, rows fitted so far). On a GPU the running totals are copied to pinned
        memory behind the tick's round and read once the copy has landed — a tick never
        waits for its own or the previous tick's round (waiting for the previous one made
        the host and the GPU take turns; see LC_LAG)."""
        cum = self.learner.cum
        if cum.device.type != "cuda":
            self._lc_point(cum.tolist())
            return
        self._lc_drain(block_over=self.LC_LAG - 1)
        host = self._lc_free.pop() if self._lc_free else None
        if host is None or host.shape != cum.shape:
            host = torch.empty(cum.shape, dtype=cum.dtype, pin_memory=True)
        host.copy_(cum, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._lc_pending.append((ev, host))

    def _lc_drain(self, block_over: int) -> None:
        """Take in the points whose copies have landed, oldest first (their order is the
        curve's); wait only while more than ``block_over`` are still in flight."""
        q = self._lc_pending
        while q:
            ev, host = q[0]
            if len(q) <= block_over and not ev.query():
                break
            ev.synchronize()
            q.popleft()
            self._lc_point(host.tolist())
            self._lc_free.append(host)

    def flush_learning_curve(self) -> None:
        """Takes every pending point in (before the curve is read or saved)."""
        self._lc_drain(block_over=0)

    def _lc_point(self, c: list) -> None:
        loss, n = c[0], int(c[1])
        dl, dn = loss - self._lc_last[0], n - self._lc_last[1]
        if dn > 0:
            self.learning_curve.append((dl / dn, n))
            self._lc_last = (loss, n)

    def update(self, request: Request) -> None:
        """Reference Update is a no-op (FlinkSpoke.scala:158); here it updates the
        learner's hyper-parameters (documented extension)."""
        if request.learner is not None and request.learner.hyperParameters:
            self.learner.update_hyper(request.learner.hyperParameters)

    # --------------------------------------------------------------- checkpoint
    def state_dict(self) -> dict:
        self.protocol.finalize()
        self.flush_learning_curve()
        return {"request": self.request.to_obj(), "learner": self.learner.state_dict(),
                "preprocessors": [p.state_dict() for p in self.preprocessors],
                "protocol": self.protocol.state_dict(),
                "learning_curve": list(self.learning_curve),
                "buffer": [self._buf_sum, self._buf_rounds]}

    def load_state_dict(self, sd: dict) -> None:
        self.learner.load_state_dict(sd["learner"])
        for p, s in zip(self.preprocessors, sd.get("preprocessors", [])):
            p.load_state_dict(s)
        self.protocol.load_state_dict(sd.get("protocol", {}))
        self.learning_curve = [tuple(x) for x in sd.get("learning_curve", [])]
        # the next learning-curve point covers the ticks after the restore, not all history
        tot = self.learner.running_totals()
        self._lc_last = (float(tot["loss_sum"]), int(tot["fitted"]))
        if sd.get("buffer"):
            self._buf_sum, self._buf_rounds = float(sd["buffer"][0]), int(sd["buffer"][1])
