"""Several pipelines in one launch (BASELINE config 5: concurrent classifiers on one stream;
reference FlinkSpoke.scala:97,101,105 feeds every point to every pipeline).

csrc/kernels/linear_scan3.hip runs M hashed-linear pipelines that share a prep as ONE
role-major launch (ops.linear.linear_scan3_round_multi); each pipeline must end exactly as
its own round would leave it, in the ops layer and through the engine."""
import json
import uuid

import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_json_records, synth_raw
from omldm_amd.ops import linear as L
from omldm_amd.ops import native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,S,R", [(1, 16, 2048), (3, 5, 700), (16, 16, 1024)])
def test_multi_pipeline_launch_matches_single_rounds(M, S, R):
    from omldm_amd.models.base import RoundContext
    from omldm_amd.models.linear import SVM, LinearLearner
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.parallel.protocols import Synchronous

    dev = torch.device("cuda", 0)
    space = FeatureSpace(13, 0, 26, 1 << 20)
    B = S * R - 5
    Cs = [0.3 + 0.1 * m for m in range(M)]
    single, multi = [], []
    for C in Cs:
        lrn = SVM({"variant": "PA-I", "C": C}, space, dev)
        proto = Synchronous(Comm(), lrn, {"virtualSpokes": S})
        for k in range(2):
            proto.round(synth_raw(space, B, start=k * B, seed=41).to(dev))
        single.append(lrn)
    learners = [SVM({"variant": "PA-I", "C": C}, space, dev) for C in Cs]
    ctx = RoundContext(spokes=S, inv_p=1.0, fused_delta=False)
    n0 = L.SCAN3_ROUNDS
    for k in range(2):
        b = synth_raw(space, B, start=k * B, seed=41).to(dev)
        assert len({lr.group_key(b, ctx) for lr in learners}) == 1
        LinearLearner.fit_group(learners, b, ctx)
    torch.cuda.synchronize()
    assert L.SCAN3_ROUNDS - n0 == 2  # one launch per round for all M pipelines
    assert native.hip().omldm_scan3_comb_err() == 0
    for a, b_ in zip(single, learners):
        d = (a.w.cpu() - b_.w.cpu()).abs()
        assert float(d.max()) < 1e-4, float(d.max())
        assert a.running_totals()["fitted"] == b_.running_totals()["fitted"] == 2 * B
        assert abs(a.running_totals()["mistakes"] - b_.running_totals()["mistakes"]) <= 2


def _job(extra=()):
    from omldm_amd.engine.job import Job
    from omldm_amd.io.transport import MemoryBroker
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.utils.config import JobConfig

    name = uuid.uuid4().hex
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", f"memory://{name}"]
    args += ["--hashDim", str(1 << 18), "--batchSize", "4096", "--parallelism", "8",
             "--timeout", "300", *extra]
    cfg = JobConfig.from_args(args)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 2)
    return Job(cfg, Comm(), "cuda"), br


def test_engine_fuses_linear_pipelines_into_one_launch():
    """Four SVM pipelines (different C) + a PA: with fusePipelines the five train in one
    launch per tick; their models equal the unfused job's."""
    models = {}
    for fuse in ("true", "false"):
        job, br = _job(["--fusePipelines", fuse])
        for pid, (name, C) in enumerate([("SVM", 0.5), ("SVM", 1.0), ("SVM", 2.0), ("PA", 1.0),
                                         ("SVM", 0.7)], start=1):
            br.produce("requests", json.dumps({
                "id": pid, "request": "Create",
                "learner": {"name": name, "hyperParameters": {"C": C}},
                "trainingConfiguration": {"protocol": "Synchronous"}}))
        sp = job.space
        for r in synth_json_records(3 * 4096, FeatureSpace(13, 0, 26, sp.dim, field_aware=True)):
            br.produce("trainingData", r)
        n0 = L.SCAN3_ROUNDS
        for _ in range(4):
            job.tick()
        torch.cuda.synchronize()
        rounds = L.SCAN3_ROUNDS - n0
        assert rounds == (3 if fuse == "true" else 15), rounds
        models[fuse] = {pid: p.learner.w.cpu().clone() for pid, p in job.pipes.items()}
        if job.fserver is not None:
            job.fserver.close()
    for pid in models["true"]:
        d = (models["true"][pid] - models["false"][pid]).abs()
        assert float(d.max()) < 1e-4, (pid, float(d.max()))


def test_logistic_pipelines_share_a_launch_only_at_equal_learning_rates():
    """The logistic prep folds lr·y into its Gram columns: pipelines with different
    learning rates need their own preps, so they never form one fused group (a mixed group
    failed the one-launch assertion in the config-5 engine run)."""
    from omldm_amd.api.batch import FeatureSpace
    from omldm_amd.io.synthetic import synth_raw
    from omldm_amd.models.base import RoundContext
    from omldm_amd.models.linear import LogisticRegression

    dev = torch.device("cuda", 0)
    space = FeatureSpace(13, 0, 26, 1 << 16)
    b = synth_raw(space, 16 * 256, seed=4).to(dev)
    ctx = RoundContext(spokes=16, inv_p=1.0, fused_delta=True)
    ks = [LogisticRegression({"learningRate": lr}, space, dev).group_key(b, ctx)
          for lr in (0.05, 0.05, 0.2)]
    assert ks[0] is not None and ks[0] == ks[1] and ks[0] != ks[2]
