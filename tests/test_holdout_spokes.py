"""Per-spoke holdout test sets and spoke-level query averaging, against a golden model of
the reference spoke.

Reference: every spoke keeps its own counter and FIFO test set of ``testSetSize``
(omldm/operators/spoke/FlinkSpoke.scala:38-41,95-104); a query scores each spoke's test
set (:136-138,160-163) and ResponseConstructor averages the P spoke answers
(omldm/utils/ResponseConstructor.scala:32-52).
"""
import json
import uuid

import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.engine.holdout import HoldoutSet
from omldm_amd.engine import statistics as ST
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.dataset import DataSet

SP = FeatureSpace(3, 1, 5, 1 << 16, field_aware=True)


class GoldenSpoke:
    """FlinkSpoke.handleData for training points, one point at a time."""

    def __init__(self, size):
        self.count = 0
        self.test = DataSet(size)
        self.trained = []

    def handle(self, point):
        if self.count >= 8:
            ev = self.test.append(point)
            if ev is not None:
                self.trained.append(ev)
        else:
            self.trained.append(point)
        self.count = (self.count + 1) % 10


def _batch(B, base, dev="cpu"):
    """Row i carries its stream id in y (and in num[:, 0]) so rows can be traced."""
    ids = torch.arange(base, base + B, dtype=torch.float32)
    num = ids.unsqueeze(1).repeat(1, SP.dn)
    cat = (torch.arange(B * SP.dc, dtype=torch.int32).view(B, SP.dc) % 30000).to(SP.cat_dtype)
    return HashedBatch(num.to(dev), cat.to(dev), ids.to(dev), cat_span=SP.cat_span)


def _run_against_golden(h: HoldoutSet, ticks, dev="cpu"):
    S, size = h.spokes, h.size
    gold = [GoldenSpoke(size) for _ in range(S)]
    base = 0
    for B in ticks:
        b = _batch(B, base, dev)
        ids = np.arange(base, base + B)
        base += B
        out = h.route(b)
        assert out.shards is not None and len(out.shards) == S and sum(out.shards) == out.B
        y = out.y.cpu().numpy()
        o = 0
        for s, (a, e) in enumerate(h.shard_bounds(B)):
            g = gold[s]
            before = len(g.trained)
            for i in ids[a:e]:
                g.handle(int(i))
            want = g.trained[before:]
            got = y[o:o + out.shards[s]]
            o += out.shards[s]
            # the spoke trains exactly the reference spoke's points (evictions are
            # trained after the shard's non-held rows instead of interleaved)
            assert sorted(got.astype(np.int64).tolist()) == sorted(want), (B, s)
        for s, t in enumerate(h.test_sets()):
            assert t.y.cpu().numpy().astype(np.int64).tolist() == gold[s].test.data_buffer, s
        assert h.n_test == sum(g.test.length for g in gold)
    return gold


def test_sixteen_spokes_route_like_sixteen_reference_spokes():
    """S = 16 spokes × testSetSize 256: every spoke's counter, FIFO and evictions match a
    reference spoke fed the same shard; the rank holds 16 × 256 test points."""
    h = HoldoutSet(SP, 256, "cpu", spokes=16)
    rng = np.random.default_rng(0)
    ticks = [65536, 4096, 17, 1000, 16 * 333, 7, 65536] + [int(v) for v in
                                                          rng.integers(1, 5000, 6)]
    _run_against_golden(h, ticks)
    assert h.n_test == 16 * 256
    assert (h.filled == 256).all()


@pytest.mark.parametrize("S,size", [(1, 4), (3, 7), (5, 1)])
def test_small_rings_and_uneven_shards(S, size):
    h = HoldoutSet(SP, size, "cpu", spokes=S)
    _run_against_golden(h, [1, 2, 9, 10, 11, 37, 200, 3, 64])


def test_spoke_padded_layout_trains_each_row_on_its_spoke():
    """Unequal shards (a short tick) are laid out as S × max(shards) for the round, so
    R-row sharding keeps every spoke's rows on that spoke; blanks are unlabeled."""
    h = HoldoutSet(SP, 8, "cpu", spokes=4)
    h.route(_batch(40, 0))
    out = h.route(_batch(13, 40))           # shards of 4, 4, 4, 1 rows in
    sh = out.shards
    pad = out.spoke_padded(4)
    R = max(sh)
    assert pad.B == 4 * R and pad.shards == (R,) * 4
    y = pad.y.numpy()
    o = 0
    for s, n in enumerate(sh):
        assert np.array_equal(y[s * R:s * R + n], out.y.numpy()[o:o + n])
        assert np.isnan(y[s * R + n:(s + 1) * R]).all()
        o += n
    assert (pad.cat.numpy()[np.isnan(y)] == -1).all()
    eq = HashedBatch(out.num, out.cat, out.y, None, out.cat_span)
    eq.shards = (3, 3, 3, 3) if out.B == 12 else None
    assert eq.spoke_padded(4) is eq


def test_state_dict_roundtrip_and_respoke():
    h = HoldoutSet(SP, 16, "cpu", spokes=4)
    for k in range(5):
        h.route(_batch(100, 100 * k))
    sd = h.state_dict()
    h2 = HoldoutSet(SP, 16, "cpu", spokes=4)
    assert h2.load_state_dict(sd) is None
    for a, b in zip(h.test_sets(), h2.test_sets()):
        assert torch.equal(a.y, b.y)
    assert np.array_equal(h.count, h2.count)
    # onto 2 spokes: old spokes 0, 2 → new 0; 1, 3 → new 1; overflow returned
    h3 = HoldoutSet(SP, 16, "cpu", spokes=2)
    spill = h3.load_state_dict(sd)
    assert h3.n_test == 32 and spill is not None and spill.B == h.n_test - 32
    old = [t.y.tolist() for t in h.test_sets()]
    assert h3.test_sets()[0].y.tolist() == (old[0] + old[2])[-16:]
    # a pre-spoke checkpoint (one ring, scalar counters) loads as one old spoke
    legacy = {"num": sd["num"][:16], "cat": sd["cat"][:16], "y": sd["y"][:16],
              "count": 3, "head": int(sd["head"][0]), "filled": int(sd["filled"][0])}
    h4 = HoldoutSet(SP, 16, "cpu", spokes=1)
    assert h4.load_state_dict(legacy) is None
    assert h4.test_sets()[0].y.tolist() == old[0]


def test_response_constructor_averages_over_spokes():
    """Loss / score: the mean of the answering spokes' values; cumulative loss and the
    mean buffer size over all spokes; dataFitted summed."""
    answers = [(0.5, 0.75, 10), (0.25, 1.0, 4), (1.0, 0.5, 2)]
    m = ST.reduce_query_metrics(Comm(), answers, fitted=100, cum_loss=30.0, mean_buffer=2.0,
                                spokes=4)
    assert m["loss"] == pytest.approx((0.5 + 0.25 + 1.0) / 3)
    assert m["score"] == pytest.approx((0.75 + 1.0 + 0.5) / 3)
    assert m["workers"] == 3 and m["spokes"] == 4 and m["testPoints"] == 16
    assert m["cumulativeLoss"] == pytest.approx(0.3)
    assert m["dataFitted"] == 100 and m["meanBufferSize"] == pytest.approx(2.0)


def test_engine_query_scores_every_spoke_test_set():
    """A 16-spoke job: the query's score is the mean of the 16 spokes' accuracies on
    their own test sets (not the pooled accuracy), and every spoke holds its ring."""
    from omldm_amd.engine.job import Job
    from omldm_amd.io.synthetic import synth_json_records
    from omldm_amd.io.transport import MemoryBroker
    from omldm_amd.utils.config import JobConfig

    name = uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(1 << 16), "--batchSize", "4000", "--timeout", "200",
             "--parallelism", "16", "--testSetSize", "32"]
    cfg = JobConfig.from_args(args)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 1)
    job = Job(cfg, Comm(), "cpu")
    space = FeatureSpace(13, 0, 26, 1 << 16)
    for r in synth_json_records(8000, space):
        br.produce("trainingData", r)
    br.produce("requests", json.dumps({"id": 1, "request": "Create",
                                       "learner": {"name": "PA", "hyperParameters": {}},
                                       "trainingConfiguration": {"protocol": "Synchronous"}}))
    for _ in range(3):
        job.tick()
    assert job.holdout.spokes == 16 and (job.holdout.filled == 32).all()
    pipe = job.pipes[1]
    accs = []
    for t in job.holdout.test_sets():
        s = pipe.learner.decision(t)
        accs.append(float(((s >= 0).float() * 2 - 1 == t.y).float().mean()))
    m = job._answer(type("Q", (), {"id": 1, "requestId": 7})(), write=False)
    assert m["spokes"] == 16 and m["workers"] == 16 and m["testPoints"] == 16 * 32
    assert m["score"] == pytest.approx(float(np.mean(accs)), abs=1e-9)
