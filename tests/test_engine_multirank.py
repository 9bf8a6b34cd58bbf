"""The whole engine on two ranks (gloo, CPU, one process per rank via the supervisor):
eight pipelines at once — every learner, every distributed protocol, preprocessors, both
categorical wires — fed from file topics, with forecasts and queries, until the idle
timeout ends the job. Checks the performance record and the outputs every rank wrote."""
import json
import os
import socket

import pytest

from omldm_amd import launch
from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import Consumer, FileBroker

PIPES = [  # id, learner, protocol, preprocessors, hyper
    (1, "SVM", "Synchronous", [], {}),
    (2, "MultiClassPA", "Asynchronous", ["StandardScaler"], {"nClasses": 2}),
    (3, "ORR", "FGM", ["PolynomialFeatures"], {}),
    (4, "NN", "SSP", ["MinMaxScaler"], {"hiddenLayers": [8]}),
    (5, "K-means", "Synchronous", [], {"k": 3}),       # forced to SingleLearner
    (6, "HT", "Asynchronous", [], {"nClasses": 2}),    # forced to SingleLearner
    (7, "RegressorPA", "EASGD", [], {}),
    (8, "PA", "GM", ["StandardScaler"], {}),
]


PIPES_ALT = [  # the same learners under other protocols (non-fused Synchronous rounds)
    (1, "SVM", "FGM", [], {}),
    (2, "MultiClassPA", "Synchronous", [], {"nClasses": 2}),
    (3, "ORR", "Synchronous", ["StandardScaler"], {}),
    (4, "NN", "Synchronous", [], {"hiddenLayers": [8]}),
    (5, "K-means", "FGM", ["MinMaxScaler"], {"k": 2}),
    (6, "HT", "Synchronous", [], {"nClasses": 2}),
    (7, "RegressorPA", "SSP", [], {}),
    (8, "PA", "EASGD", [], {}),
]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
@pytest.mark.parametrize("field_aware", [False, True])
def test_two_rank_job_every_learner_and_protocol(tmp_path, field_aware):
    _two_rank_job(tmp_path, field_aware, "cpu")


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("field_aware", [False, True])
def test_two_rank_job_every_learner_and_protocol_gpu(tmp_path, field_aware):
    """The same job with both ranks on the one GPU of the box (HIP kernels, device-resident
    state; the two ranks talk over gloo — the 8-GPU RCCL run is the driver's)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _two_rank_job(tmp_path, field_aware, "cuda", {"OMLDM_DIST_BACKEND": "gloo"})


def _two_rank_job(tmp_path, field_aware, device, env=None):
    data = tmp_path / "topics"
    br = FileBroker(str(data))
    sp = FeatureSpace(5, 0, 6, 1 << 14, field_aware=field_aware)
    br.create_topic("trainingData", 4)
    br.create_topic("forecastingData", 2)
    for i, r in enumerate(synth_json_records(3000, sp, seed=5)):
        br.produce("trainingData", r, partition=i % 4)
    for i, r in enumerate(synth_json_records(10, sp, seed=6, operation="forecasting")):
        br.produce("forecastingData", r, partition=i % 2)
    for pid, learner, proto, pre, hyper in PIPES:
        br.produce("requests", json.dumps({
            "id": pid, "request": "Create", "learner": {"name": learner, "hyperParameters": hyper},
            "preProcessors": [{"name": p} for p in pre],
            "trainingConfiguration": {"protocol": proto}}))
    for pid, *_ in PIPES:
        br.produce("requests", json.dumps({"id": pid, "request": "Query", "requestId": 500 + pid}))
    # lifecycle on every rank: pipeline 9 created, updated, deleted, re-created as another
    # learner (its final statistics must be the new learner's)
    for req in ({"id": 9, "request": "Create", "learner": {"name": "SVM"},
                 "trainingConfiguration": {"protocol": "Synchronous"}},
                {"id": 9, "request": "Update", "learner": {"name": "SVM",
                                                            "hyperParameters": {"C": 0.1}}},
                {"id": 9, "request": "Delete"},
                {"id": 9, "request": "Create", "learner": {"name": "RegressorPA"},
                 "trainingConfiguration": {"protocol": "Asynchronous"}}):
        br.produce("requests", json.dumps(req))
    addr = f"file://{data}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(sp.dim), "--numFeatures", "5", "--catFeatures", "6",
             "--fieldAware", str(field_aware).lower(), "--device", device, "--batchSize", "250",
             "--timeout", "1500", "--parallelism", "4", "--jobName", "two-rank",
             "--parseThreads", "2", "--watchdogTimeout", "120000"]
    env_before = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ.update(env or {})
    try:
        logs = []
        rc = launch.supervise(2, args, max_restarts=0, min_nproc=2, port=_port(), log=logs.append)
    finally:
        os.environ.clear()
        os.environ.update(env_before)
    assert rc == 0, logs
    js = json.loads(Consumer(br, "performance", all_partitions=True).poll(10)[-1])
    assert js["jobName"] == "two-rank" and js["metrics"]["ranks"] == 2
    assert js["parallelism"] == 2 * js["metrics"]["spokesPerRank"]
    stats = {s["pipeline"]: s for s in js["statistics"]}
    assert sorted(stats) == [p[0] for p in PIPES] + [9]
    assert stats[9]["protocol"] == "Asynchronous" and stats[9]["fitted"] > 0
    for pid, learner, proto, _, _ in PIPES:
        st = stats[pid]
        assert st["fitted"] > 0, (pid, st)
        want = "SingleLearner" if learner in ("K-means", "HT") else proto
        assert st["protocol"] == want, (pid, st["protocol"])
    preds = [json.loads(x) for x in Consumer(br, "predictions", all_partitions=True).poll(1000)]
    assert len(preds) == 10 * (len(PIPES) + 1)
    assert {p["mlpId"] for p in preds} == {p[0] for p in PIPES} | {9}
    # one reduced answer per query (the final, non-bucket response carries the metrics)
    resp = [json.loads(x) for x in Consumer(br, "responses", all_partitions=True).poll(10000)]
    finals = [r for r in resp if r.get("responseId", -1) >= 500 and r.get("loss") is not None]
    assert sorted(r["responseId"] for r in finals) == [500 + p[0] for p in PIPES]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("pipes", [PIPES, PIPES_ALT], ids=["protocols", "protocols_alt"])
def test_two_rank_job_killed_and_restored_on_one_rank(tmp_path, pipes):
    """Checkpoint every tick, rank 1 killed at tick 6, the supervisor restarts the job on
    one rank from the last checkpoint: every learner's and protocol's state goes through
    a re-scaled restore (2 → 1 ranks) and the job finishes with all eight pipelines."""
    _kill_restore(tmp_path, pipes, "cpu")


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("pipes", [PIPES, PIPES_ALT], ids=["protocols", "protocols_alt"])
def test_two_rank_job_killed_and_restored_on_one_rank_gpu(tmp_path, pipes):
    """The same with device-resident learner state (HBM models, shadows, the HT tree)
    checkpointed from and restored onto the GPU."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _kill_restore(tmp_path, pipes, "cuda", {"OMLDM_DIST_BACKEND": "gloo"})


def _kill_restore(tmp_path, pipes, device, env=None):
    data = tmp_path / "topics"
    br = FileBroker(str(data))
    sp = FeatureSpace(5, 0, 6, 1 << 14, field_aware=True)
    br.create_topic("trainingData", 4)
    for i, r in enumerate(synth_json_records(4000, sp, seed=7)):
        br.produce("trainingData", r, partition=i % 4)
    for pid, learner, proto, pre, hyper in pipes:
        br.produce("requests", json.dumps({
            "id": pid, "request": "Create", "learner": {"name": learner, "hyperParameters": hyper},
            "preProcessors": [{"name": p} for p in pre],
            "trainingConfiguration": {"protocol": proto, "HubParallelism": 1}}))
    addr = f"file://{data}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(sp.dim), "--numFeatures", "5", "--catFeatures", "6",
             "--fieldAware", "true", "--device", device, "--batchSize", "200",
             "--timeout", "1500", "--parallelism", "4", "--jobName", "restore-all",
             "--checkpointing", "true", "--checkInterval", "0",
             "--stateBackend", str(tmp_path / "ckpt"), "--faults", "kill:rank=1:tick=6",
             "--parseThreads", "2", "--watchdogTimeout", "120000"]
    env_before = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ.update(env or {})
    try:
        logs = []
        rc = launch.supervise(2, args, max_restarts=2, min_nproc=1, shrink=True, port=_port(),
                              log=logs.append)
    finally:
        os.environ.clear()
        os.environ.update(env_before)
    assert rc == 0, logs
    assert any("on 1 rank(s)" in m for m in logs), logs
    js = json.loads(Consumer(br, "performance", all_partitions=True).poll(10)[-1])
    assert js["jobName"] == "restore-all" and js["metrics"]["ranks"] == 1
    assert js["parallelism"] == 1 * js["metrics"]["spokesPerRank"]
    stats = {s["pipeline"]: s for s in js["statistics"]}
    assert sorted(stats) == [p[0] for p in pipes]
    for pid, learner, proto, _, _ in pipes:
        assert stats[pid]["fitted"] > 0, (pid, stats[pid])


@pytest.mark.timeout(300)
def test_two_rank_job_over_kafka_with_compressed_topics(tmp_path):
    """Two ranks consuming and producing through the Kafka wire client against the
    protocol-level fake broker: lz4-compressed input batches, zstd-compressed outputs
    (Produce v7 / Fetch v10 negotiated), every rank reading its share of the partitions."""
    from omldm_amd.io.kafka import KafkaBroker
    from tests.fake_kafka import FakeKafka

    fk = FakeKafka(default_partitions=4)
    try:
        sp = FeatureSpace(5, 0, 6, 1 << 14, field_aware=True)
        src = KafkaBroker(f"{fk.addr}?compression=lz4")
        for t in ("trainingData", "forecastingData", "requests", "responses", "predictions",
                  "performance"):
            src.create_topic(t, 1 if t in ("requests", "responses", "performance") else 4)
        recs = [r.encode() for r in synth_json_records(2000, sp, seed=9)]
        for p in range(4):
            src.produce_batch("trainingData", p, recs[p::4])
        src.produce_batch("forecastingData", 0, [r.encode() for r in synth_json_records(
            6, sp, seed=10, operation="forecasting")])
        for pid, learner, proto, pre, hyper in PIPES[:4]:
            src.produce("requests", json.dumps({
                "id": pid, "request": "Create",
                "learner": {"name": learner, "hyperParameters": hyper},
                "preProcessors": [{"name": p} for p in pre],
                "trainingConfiguration": {"protocol": proto}}), partition=0)
        out = f"{fk.addr}?compression=zstd"
        args = ["--trainingDataAddr", fk.addr, "--forecastingDataAddr", fk.addr,
                "--requestsAddr", fk.addr, "--responsesAddr", out, "--predictionsAddr", out,
                "--performanceAddr", out,
                "--hashDim", str(sp.dim), "--numFeatures", "5", "--catFeatures", "6",
                "--fieldAware", "true", "--device", "cpu", "--batchSize", "200",
                "--timeout", "1500", "--parallelism", "4", "--jobName", "kafka-two-rank",
                "--parseThreads", "2", "--watchdogTimeout", "120000"]
        env_before = dict(os.environ)
        os.environ["OMP_NUM_THREADS"] = "1"
        try:
            logs = []
            rc = launch.supervise(2, args, max_restarts=0, min_nproc=2, port=_port(),
                                  log=logs.append)
        finally:
            os.environ.clear()
            os.environ.update(env_before)
        assert rc == 0, logs
        rd = KafkaBroker(fk.addr)
        perf, _ = rd.consume("performance", 0, 0, 10)
        js = json.loads(perf[-1])
        assert js["jobName"] == "kafka-two-rank" and js["metrics"]["ranks"] == 2
        assert js["parallelism"] == 2 * js["metrics"]["spokesPerRank"]
        assert sorted(s["pipeline"] for s in js["statistics"]) == [1, 2, 3, 4]
        assert all(s["fitted"] > 0 for s in js["statistics"])
        preds = []
        for p in range(rd.partitions("predictions")):
            v, _ = rd.consume("predictions", p, 0, 1000)
            preds += v
        assert len(preds) == 6 * 4
    finally:
        fk.close()


@pytest.mark.timeout(300)
def test_four_rank_job_mixed_hub_layouts(tmp_path):
    """Four ranks, Synchronous pipelines with HubParallelism 1 (reduce + broadcast), 2
    (sharded hubs) and 4 (all-reduce) side by side: the engine coalesces each layout's
    round buffers into its own collective (collective order must agree on every rank, or
    the job deadlocks); every pipeline trains and is reported."""
    _four_rank(tmp_path, "cpu")


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_four_rank_job_mixed_hub_layouts_gpu(tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _four_rank(tmp_path, "cuda", {"OMLDM_DIST_BACKEND": "gloo"})


def _four_rank(tmp_path, device, env=None):
    data = tmp_path / "topics"
    br = FileBroker(str(data))
    sp = FeatureSpace(5, 0, 6, 1 << 14, field_aware=True)
    br.create_topic("trainingData", 4)
    for i, r in enumerate(synth_json_records(3200, sp, seed=11)):
        br.produce("trainingData", r, partition=i % 4)
    layouts = {1: ("SVM", 1), 2: ("PA", 2), 3: ("RegressorPA", 4), 4: ("ORR", 2), 5: ("NN", 1)}
    for pid, (learner, hubs) in layouts.items():
        br.produce("requests", json.dumps({
            "id": pid, "request": "Create",
            "learner": {"name": learner,
                        "hyperParameters": {"hiddenLayers": [8]} if learner == "NN" else {}},
            "trainingConfiguration": {"protocol": "Synchronous", "HubParallelism": hubs}}))
    for pid in layouts:
        br.produce("requests", json.dumps({"id": pid, "request": "Query", "requestId": 100 + pid}))
    addr = f"file://{data}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(sp.dim), "--numFeatures", "5", "--catFeatures", "6",
             "--fieldAware", "true", "--device", device, "--batchSize", "200",
             "--timeout", "1500", "--parallelism", "8", "--jobName", "hubs",
             "--parseThreads", "1", "--watchdogTimeout", "120000"]
    env_before = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ.update(env or {})
    try:
        logs = []
        rc = launch.supervise(4, args, max_restarts=0, min_nproc=4, port=_port(), log=logs.append)
    finally:
        os.environ.clear()
        os.environ.update(env_before)
    assert rc == 0, logs
    js = json.loads(Consumer(br, "performance", all_partitions=True).poll(10)[-1])
    assert js["metrics"]["ranks"] == 4
    assert js["parallelism"] == 4 * js["metrics"]["spokesPerRank"]
    stats = {s["pipeline"]: s for s in js["statistics"]}
    assert sorted(stats) == sorted(layouts)
    assert all(s["fitted"] > 0 and s["protocol"] == "Synchronous" for s in stats.values())


@pytest.mark.timeout(300)
def test_restore_grows_from_one_rank_to_two(tmp_path):
    """A one-rank job checkpoints and stops after a few ticks; the job is restarted with
    --restore on two ranks (the re-scaled restore growing the world): every learner's
    state, the pipelines and the consumer offsets carry over and the job completes."""
    data = tmp_path / "topics"
    br = FileBroker(str(data))
    sp = FeatureSpace(5, 0, 6, 1 << 14, field_aware=True)
    br.create_topic("trainingData", 4)
    for i, r in enumerate(synth_json_records(4000, sp, seed=13)):
        br.produce("trainingData", r, partition=i % 4)
    for pid, learner, proto, pre, hyper in PIPES:
        br.produce("requests", json.dumps({
            "id": pid, "request": "Create", "learner": {"name": learner, "hyperParameters": hyper},
            "preProcessors": [{"name": p} for p in pre],
            "trainingConfiguration": {"protocol": proto}}))
    addr = f"file://{data}"
    base = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        base += [f"--{k}", addr]
    base += ["--hashDim", str(sp.dim), "--numFeatures", "5", "--catFeatures", "6",
             "--fieldAware", "true", "--device", "cpu", "--batchSize", "200",
             "--timeout", "1500", "--parallelism", "4", "--jobName", "grow",
             "--checkpointing", "true", "--checkInterval", "0",
             "--stateBackend", str(tmp_path / "ckpt"), "--parseThreads", "2",
             "--watchdogTimeout", "120000"]
    env_before = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        logs = []
        rc = launch.supervise(1, base + ["--maxTicks", "6"], max_restarts=0, min_nproc=1,
                              port=_port(), log=logs.append)
        assert rc == 0, logs
        assert not Consumer(br, "performance", all_partitions=True).poll(10)  # not finished
        rc = launch.supervise(2, base + ["--restore", "true"], max_restarts=0, min_nproc=2,
                              port=_port(), log=logs.append)
    finally:
        os.environ.clear()
        os.environ.update(env_before)
    assert rc == 0, logs
    js = json.loads(Consumer(br, "performance", all_partitions=True).poll(10)[-1])
    assert js["jobName"] == "grow" and js["metrics"]["ranks"] == 2
    assert js["parallelism"] == 2 * js["metrics"]["spokesPerRank"]
    # the restored consumer offsets: the second run trained only on what the first did
    # not consume (a fresh start would re-train on all ≈ 0.8 × 4000 rows)
    assert js["metrics"]["trainedExamples"] < 2900, js["metrics"]["trainedExamples"]
    stats = {s["pipeline"]: s for s in js["statistics"]}
    assert sorted(stats) == [p[0] for p in PIPES]
    assert all(s["fitted"] > 0 for s in stats.values())
