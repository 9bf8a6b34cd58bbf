"""Statistics parity with the reference's StatisticsOperator / StateAccumulators.

* meanBufferSize: the −1 query carries each spoke's mean buffer size / P and the operator
  sums them (FlinkSpoke.scala:136-138, StatisticsOperator.scala:101) — the mean over
  spokes of the records a spoke holds when its round starts;
* JobStatistics.parallelism is the spoke parallelism (StatisticsOperator.scala:109-113);
* a pipeline's H hub records are summed, then blocks / models / fitted divided by H
  (StateAccumulators.scala:94-108) — bytes stay summed.
"""
import json
import uuid

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.engine.job import Job
from omldm_amd.engine.statistics import merge_hub_statistics
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import MemoryBroker
from omldm_amd.models import make_learner
from omldm_amd.parallel.comm import Comm
from omldm_amd.parallel.protocols import Synchronous
from omldm_amd.utils.config import JobConfig

SP = FeatureSpace(13, 0, 26, 1 << 14)


def test_hub_merge_rule():
    hubs = [{"modelsShipped": 8, "bytesShipped": 100, "numOfBlocks": 6},
            {"modelsShipped": 8, "bytesShipped": 50, "numOfBlocks": 4}]
    m = merge_hub_statistics(hubs, fitted=1000)
    assert m == {"modelsShipped": 8, "bytesShipped": 150, "numOfBlocks": 5, "fitted": 1000,
                 "hubs": 2}


class _FakeComm(Comm):
    def __init__(self, world):
        super().__init__()
        self.world, self.rank, self.backend = world, 0, "gloo"


def test_per_hub_blocks_follow_the_shards():
    """H = 2 hubs of 4 workers, 25,000 parameters, 10,000 per block: each hub's shard is
    12,500 parameters = 2 blocks per message, 2·4 messages per sync."""
    L = make_learner("PA", {}, SP, "cpu")
    P = Synchronous(_FakeComm(4), L, {"HubParallelism": 2}, max_msg_params=10000)
    P._account_model_sync(25000, 100000)
    P._account_model_sync(25000, 100000)
    hs = P.hub_statistics()
    assert len(hs) == 2
    assert all(h["modelsShipped"] == 16 and h["numOfBlocks"] == 32 for h in hs)
    assert sum(h["bytesShipped"] for h in hs) == 2 * 2 * 4 * 100000
    m = merge_hub_statistics(hs, 0)
    assert m["numOfBlocks"] == 32 and m["modelsShipped"] == 16
    # one hub (every rank a hub when H = 0: G shards)
    P1 = Synchronous(_FakeComm(4), L, {"HubParallelism": 1}, max_msg_params=10000)
    P1._account_model_sync(25000, 100000)
    assert P1.hub_statistics() == [{"modelsShipped": 8, "bytesShipped": 800000,
                                    "numOfBlocks": 24}]
    P0 = Synchronous(_FakeComm(4), L, {}, max_msg_params=10000)
    assert P0.n_hubs() == 4


def test_job_statistics_spoke_parallelism_and_mean_buffer_size():
    name = uuid.uuid4().hex
    addr = f"memory://{name}"
    args = []
    for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
              "predictionsAddr", "performanceAddr"):
        args += [f"--{k}", addr]
    args += ["--hashDim", str(SP.dim), "--batchSize", "400", "--timeout", "200",
             "--parallelism", "4", "--testSetSize", "64"]
    cfg = JobConfig.from_args(args)
    br = MemoryBroker.named(name)
    br.create_topic(cfg.trainingDataTopic, 1)
    br.produce("requests", json.dumps({"id": 1, "request": "Create",
                                       "learner": {"name": "SVM"},
                                       "trainingConfiguration": {"protocol": "Synchronous"}}))
    for r in synth_json_records(2000, SP):
        br.produce("trainingData", r)
    job = Job(cfg, Comm(), "cpu")
    job.run()
    perf = json.loads(br.records("performance")[-1])
    assert perf["parallelism"] == 4 == job.spokes * job.world
    st = perf["statistics"][0]
    # 400-record ticks, 2/10 of the routed rows held out → training rounds of ≈ 320 rows
    # over 4 spokes: ≈ 80 records per spoke per round (the first tick's rows fill the
    # holdout ring first)
    assert 40.0 <= st["meanBufferSize"] <= 100.0, st
    assert st["extra"]["hubs"] == 1 and st["fitted"] > 0
    # engine-internal hyper-parameters never reach a response
    assert all(not k.startswith("_") for k in job.pipes[1].learner.hyper_parameters())


def test_synthetic_json_is_reproducible_across_processes():
    import subprocess
    import sys

    code = ("from omldm_amd.api.batch import FeatureSpace;"
            "from omldm_amd.io.synthetic import synth_json_records;"
            "print(synth_json_records(50, FeatureSpace(13, 0, 26, 1 << 14))[-1])")
    outs = set()
    for hs in ("1", "2", "random"):
        env = {**__import__("os").environ, "PYTHONHASHSEED": hs}
        outs.add(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True,
                                text=True, check=True).stdout)
    assert len(outs) == 1
