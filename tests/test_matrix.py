"""Configuration matrix through the whole engine (CPU, in-process broker): every reference
learner × every preprocessor × both categorical wires (global int32 hashing and the
field-aware uint16 slots). Each job creates the pipeline, trains, forecasts, answers a
query, applies an Update and a Delete — the flows a reference user drives through the
requests topic. Catches configuration-only bugs (a dropped wire flag, a learner that
cannot take a preprocessed batch) that single-path tests miss."""
import json
import math
import uuid

import pytest

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.api.schemas import VALID_LEARNERS, VALID_PREPROCESSORS
from omldm_amd.engine.job import Job
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import MemoryBroker
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.config import JobConfig

HYPER = {"MultiClassPA": {"nClasses": 3}, "K-means": {"k": 3}, "HT": {"nClasses": 3},
         "NN": {"hiddenLayers": [16]}}
TASK = {"RegressorPA": 1, "ORR": 1, "MultiClassPA": 2, "HT": 2}  # synth_json_records task


@pytest.mark.parametrize("field_aware", [False, True])
@pytest.mark.parametrize("pre", [None, *VALID_PREPROCESSORS])
@pytest.mark.parametrize("learner", VALID_LEARNERS)
def test_learner_preprocessor_wire_matrix(learner, pre, field_aware):
    _run(learner, pre, field_aware, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("field_aware", [False, True])
@pytest.mark.parametrize("pre", [None, *VALID_PREPROCESSORS])
@pytest.mark.parametrize("learner", VALID_LEARNERS)
def test_learner_preprocessor_wire_matrix_gpu(cuda, learner, pre, field_aware):
    """The same flows on the HIP kernels (GPU JSON parse, device holdout, every learner's
    round kernel, preprocessing kernels, both wires)."""
    _run(learner, pre, field_aware, cuda)


PROTOCOLS = ("CentralizedTraining", "SingleLearner", "Asynchronous", "Synchronous", "SSP",
             "EASGD", "GM", "FGM")


@pytest.mark.parametrize("protocol", PROTOCOLS)
@pytest.mark.parametrize("learner", ["SVM", "MultiClassPA", "ORR", "NN"])
def test_learner_protocol_matrix(learner, protocol):
    _run(learner, "StandardScaler", True, "cpu", protocol)


@pytest.mark.gpu
@pytest.mark.parametrize("protocol", PROTOCOLS)
@pytest.mark.parametrize("learner", ["SVM", "MultiClassPA", "ORR", "NN"])
def test_learner_protocol_matrix_gpu(cuda, learner, protocol):
    _run(learner, "StandardScaler", True, cuda, protocol)


VARIANTS = [("SVM", {"variant": "Pegasos", "lambda": 1e-3}), ("SVM", {"modelDtype": "bf16"}),
            ("PA", {"variant": "PA-II", "C": 0.5}), ("PA", {"variant": "PA"}),
            ("RegressorPA", {"variant": "PA-I", "epsilon": 0.2, "modelDtype": "bf16"}),
            ("MultiClassPA", {"nClasses": 4, "variant": "PA-II", "modelDtype": "bf16"}),
            ("NN", {"hiddenLayers": [24, 12], "activation": "tanh", "matmulDtype": "bf16"}),
            ("NN", {"hiddenLayers": [8], "activation": "sigmoid", "task": "regression"}),
            ("NN", {"hiddenLayers": [16], "nClasses": 3}),
            ("K-means", {"k": 40}), ("HT", {"nClasses": 3, "gracePeriod": 50, "nBins": 8}),
            ("ORR", {"lambda": 0.1})]


@pytest.mark.parametrize("learner,hyper", VARIANTS)
def test_learner_variants(learner, hyper):
    _run(learner, None, True, "cpu", hyper=hyper)


@pytest.mark.gpu
@pytest.mark.parametrize("learner,hyper", VARIANTS)
def test_learner_variants_gpu(cuda, learner, hyper):
    _run(learner, None, True, cuda, hyper=hyper)


@pytest.mark.parametrize("learner", ["SVM", "MultiClassPA", "ORR", "NN", "K-means", "HT"])
def test_discrete_features_and_serving_mode(learner):
    """Points with discrete features (dense slots after the numerical ones) and a job in
    serving mode (--test false: no idle termination, answers still flow)."""
    _run(learner, "MinMaxScaler", True, "cpu", discrete=2,
         extra=["--discreteFeatures", "2", "--test", "false"])


FLAGS = [["--gpuParse", "false"], ["--prefetch", "false"], ["--ingestCUs", "16"],
         ["--ingestCopy", "sdma"], ["--gpuParse", "false", "--prefetch", "false"]]


@pytest.mark.gpu
@pytest.mark.parametrize("flags", FLAGS, ids=lambda f: "_".join(x.strip("-") for x in f))
@pytest.mark.parametrize("learner", ["SVM", "MultiClassPA", "HT"])
def test_engine_ingest_flags_gpu(cuda, learner, flags):
    """Engine ingest variants on the GPU: host JSON parser instead of the GPU one, no
    read-ahead, XCD-local ingest CUs, SDMA staging copies."""
    _run(learner, "StandardScaler", True, cuda, extra=flags)


def _run(learner, pre, field_aware, device, protocol="Synchronous", hyper=None, extra=(),
         discrete=0):
    name = uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(1 << 16), "--batchSize", "400", "--timeout", "200",
             "--parallelism", "4", "--numFeatures", "5", "--catFeatures", "6",
             "--fieldAware", str(field_aware).lower(), *extra]
    cfg = JobConfig.from_args(args)
    sp = FeatureSpace(5, discrete, 6, 1 << 16, field_aware=field_aware)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 2)
    job = Job(cfg, Comm(), device)
    try:
        _drive(job, br, sp, learner, pre, protocol, hyper)
    finally:
        job.close()  # no lane thread, read-ahead or resident wave outlives the test


def _drive(job, br, sp, learner, pre, protocol, hyper):
    br.produce("requests", json.dumps({
        "id": 7, "request": "Create",
        "learner": {"name": learner, "hyperParameters": hyper or HYPER.get(learner, {})},
        "preProcessors": [{"name": pre}] if pre else [],
        "trainingConfiguration": {"protocol": protocol}}))
    for r in synth_json_records(1200, sp, task=TASK.get(learner, 0)):
        br.produce("trainingData", r)
    for _ in range(4):
        job.tick()
    assert 7 in job.pipes
    for r in synth_json_records(5, sp, start=9000, operation="forecasting",
                                task=TASK.get(learner, 0)):
        br.produce("forecastingData", r)
    br.produce("requests", json.dumps({"id": 7, "request": "Query", "requestId": 11}))
    for _ in range(3):
        job.tick()
    preds = [json.loads(x) for x in br.records("predictions")]
    assert len(preds) == 5 and all(p["mlpId"] == 7 for p in preds)
    resp = [json.loads(x) for x in br.records("responses")]
    final = [r for r in resp if r.get("responseId") == 11 and r.get("loss") is not None]
    assert final and final[-1]["dataFitted"] > 0
    for k in ("loss", "score"):
        v = final[-1].get(k)
        assert v is None or math.isfinite(float(v)), (k, v)
    br.produce("requests", json.dumps({"id": 7, "request": "Update",
                                       "learner": {"name": learner,
                                                   "hyperParameters": HYPER.get(learner, {})}}))
    job.tick()
    br.produce("requests", json.dumps({"id": 7, "request": "Delete"}))
    job.tick()
    assert 7 not in job.pipes


@pytest.mark.parametrize("protocol", ["SingleLearner", "Synchronous", "FGM"])
def test_orr_fused_polynomial_under_every_forwarding_protocol(protocol):
    """ORR + PolynomialFeatures fuses the degree-2 map into the Gram kernel (a PolyBatch
    reaches the learner); a protocol that regroups the batch must keep that kind."""
    _run("ORR", "PolynomialFeatures", True, "cpu", protocol)


def test_hostile_requests_are_dropped_not_fatal():
    """Malformed or ill-typed requests (reference: a malformed request kills the job,
    RequestParser.scala:12-16; here it is dropped and counted) next to a valid one."""
    name = uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(1 << 16), "--batchSize", "400", "--timeout", "200",
             "--parallelism", "4", "--numFeatures", "5", "--catFeatures", "6"]
    cfg = JobConfig.from_args(args)
    sp = FeatureSpace(5, 0, 6, 1 << 16)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 2)
    job = Job(cfg, Comm(), "cpu")
    hostile = [
        "not json", "[]", "{}", '{"id": 1}', '{"id": "x", "request": "Create"}',
        json.dumps({"id": 2, "request": "create", "learner": {"name": "SVM"}}),
        json.dumps({"id": 3, "request": "Create"}),
        json.dumps({"id": 4, "request": "Create", "learner": {"name": "Nope"}}),
        json.dumps({"id": 5, "request": "Create", "learner": {"name": "SVM"},
                    "preProcessors": [{"name": "Whitening"}]}),
        json.dumps({"id": 6, "request": "Create", "learner": {"name": "SVM",
                                                              "hyperParameters": [1, 2]}}),
        json.dumps({"id": 7, "request": "Create", "learner": {"name": "SVM"},
                    "trainingConfiguration": {"protocol": 42, "HubParallelism": "abc"}}),
        json.dumps({"id": 8, "request": "Create", "learner": {"name": "NN",
                                                              "hyperParameters": {"hiddenLayers": "big"}}}),
        json.dumps({"id": 9, "request": "Query"}),
        json.dumps({"id": 10, "request": "Delete"}),
        json.dumps({"id": 11, "request": "Create", "learner": {"name": "PA"},
                    "trainingConfiguration": {"protocol": "Synchronous"}}),
    ]
    for h in hostile:
        br.produce("requests", h)
    for r in synth_json_records(800, sp):
        br.produce("trainingData", r)
    for _ in range(4):
        job.tick()
    assert 11 in job.pipes  # the valid request went through
    assert not job.terminated
    br.produce("requests", json.dumps({"id": 11, "request": "Query", "requestId": 5}))
    for _ in range(2):
        job.tick()
    resp = [json.loads(x) for x in br.records("responses")]
    assert any(r.get("responseId") == 5 for r in resp)


def test_update_retunes_or_rejects():
    """Update changes tunable hyper-parameters of a live learner (learning rates, split
    thresholds, margins) and is refused for shape-fixing ones (layer widths, classes, k),
    which the engine then drops and counts (the reference's Update is a no-op)."""
    from omldm_amd.models import make_learner

    sp = FeatureSpace(5, 0, 6, 1 << 12)
    nn = make_learner("NN", {"hiddenLayers": [8]}, sp, "cpu")
    nn.update_hyper({"learningRate": 0.2, "activation": "tanh"})
    assert nn.lr == 0.2 and nn.act_name == "tanh"
    with pytest.raises(ValueError):
        nn.update_hyper({"hiddenLayers": [16]})
    ht = make_learner("HT", {"nClasses": 3}, sp, "cpu")
    ht.update_hyper({"gracePeriod": 50, "delta": 1e-3})
    assert ht.grace == 50 and ht.delta == 1e-3
    with pytest.raises(ValueError):
        ht.update_hyper({"nClasses": 4})
    mc = make_learner("MultiClassPA", {"nClasses": 3}, sp, "cpu")
    mc.update_hyper({"C": 0.25, "variant": "PA-II"})
    assert mc.C == 0.25 and mc.variant == 2
    km = make_learner("K-means", {"k": 4}, sp, "cpu")
    km.update_hyper({"k": 4})  # unchanged value: accepted
    with pytest.raises(ValueError):
        km.update_hyper({"k": 5})


def test_rejected_update_is_not_partially_applied():
    """Update {variant: Pegasos, lambda: 0} used to leave the Pegasos rule with
    λ = 0 behind (the next round failed); NN 'bogus' activation stayed in hyper."""
    import torch

    from omldm_amd.api.batch import FeatureSpace as FS
    from omldm_amd.io.synthetic import synth_batch
    from omldm_amd.models import make_learner
    from omldm_amd.models.base import RoundContext

    sp = FS(5, 0, 6, 1 << 12)
    svm = make_learner("SVM", {"variant": "PA-I"}, sp, "cpu")
    with pytest.raises(ValueError):
        svm.update_hyper({"variant": "Pegasos", "lambda": 0})
    assert svm.hyper_parameters()["variant"] == "PA-I"
    assert "lambda" not in svm.hyper or svm.hyper["lambda"] != 0
    b = synth_batch(sp, 64, seed=3)
    svm.fit(b, RoundContext(spokes=2, inv_p=0.5))  # still trains (PA-I)
    sd = svm.state_dict()
    svm2 = make_learner("SVM", {"variant": "PA-I"}, sp, "cpu")
    svm2.load_state_dict(sd)
    svm2.fit(b, RoundContext(spokes=2, inv_p=0.5))
    nn = make_learner("NN", {"hiddenLayers": [8]}, sp, "cpu")
    with pytest.raises(ValueError):
        nn.update_hyper({"activation": "bogus", "learningRate": 0.5})
    assert nn.act_name == "relu" and nn.lr == 0.05
    assert "activation" not in nn.hyper and "learningRate" not in nn.hyper
    assert torch.isfinite(nn.flat).all()


def test_restore_keeps_updated_tunables():
    """after Update → checkpoint → restore, the restored learner trains with
    the Updated settings (not Create's) for every learner kind with tunables."""
    from omldm_amd.models import make_learner

    sp = FeatureSpace(5, 0, 6, 1 << 12)
    cases = [("NN", {"hiddenLayers": [8]}, {"learningRate": 0.2, "activation": "tanh"},
              lambda m: (m.lr, m.act_name) == (0.2, "tanh")),
             ("HT", {"nClasses": 3}, {"gracePeriod": 50, "tau": 0.2},
              lambda m: (m.grace, m.tau) == (50, 0.2)),
             ("MultiClassPA", {"nClasses": 3}, {"C": 0.25, "variant": "PA-II"},
              lambda m: (m.C, m.variant) == (0.25, 2)),
             ("ORR", {}, {"lambda": 3.0}, lambda m: m.lam == 3.0),
             ("PA", {}, {"C": 0.5, "variant": "PA-II"},
              lambda m: (m.rule.C, m.rule.variant) == (0.5, 2))]
    for name, create, upd, check in cases:
        a = make_learner(name, dict(create), sp, "cpu")
        a.update_hyper(upd)
        assert check(a), name
        b = make_learner(name, dict(create), sp, "cpu")
        b.load_state_dict(a.state_dict())
        assert check(b), name


def test_structural_check_uses_values_in_use():
    """keys Create left at their default must still be refused when changed,
    and equal values in another spelling ('[8]' vs [8], '4' vs 4) are accepted."""
    from omldm_amd.models import make_learner

    sp = FeatureSpace(5, 0, 6, 1 << 12)
    nn = make_learner("NN", {}, sp, "cpu")          # hiddenLayers default [32, 32]
    with pytest.raises(ValueError):
        nn.update_hyper({"hiddenLayers": [8]})
    nn.update_hyper({"hiddenLayers": "[32, 32]"})   # same shape: accepted
    km = make_learner("K-means", {}, sp, "cpu")     # k default 8
    with pytest.raises(ValueError):
        km.update_hyper({"k": 3})
    km.update_hyper({"k": "8"})
    ht = make_learner("HT", {}, sp, "cpu")
    for k, v in (("nClasses", 5), ("maxNodes", 7), ("maxDepth", 3), ("nBins", 4)):
        with pytest.raises(ValueError):
            ht.update_hyper({k: v})
    mc = make_learner("MultiClassPA", {}, sp, "cpu")  # nClasses default 2
    with pytest.raises(ValueError):
        mc.update_hyper({"nClasses": 4})
