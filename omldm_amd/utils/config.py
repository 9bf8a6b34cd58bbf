"""Job configuration: the reference's CLI flags (same names, same defaults) + the
MI355X-native engine's own flags.

Reference flags: omldm/Job.scala:110-168 (ParameterTool.fromArgs), defaults in
omldm/utils/DefaultJobParameters.scala:4-11, omldm/utils/Checkpointing.scala:11-23,
omldm/job/FlinkLearning.scala:43-48. Accepted and ignored, with
the reason: ``psMessages*`` (the parameter-server feedback loop is RCCL / point-to-point,
not a Kafka topic) and ``local`` (the reference picks a local mini-cluster or a remote
Flink environment; here every launch is one process per GPU through omldm_amd.launch).
The reference's hub cache (StateAccumulators.scala:38) and 100-record heartbeat
(FlinkSpoke.scala:85) have no knob: hubs are collectives with no message cache, and
every tick's control all-reduce is the heartbeat.
"""
from __future__ import annotations

import argparse
from dataclasses import asdict, dataclass, field, fields


def _bool(v) -> bool:
    if isinstance(v, bool):
        return v
    return str(v).strip().lower() in ("1", "true", "yes", "y", "on")


@dataclass
class JobConfig:
    # ---- reference flags (names and defaults kept)
    parallelism: int = 16
    jobName: str = "OML_job_1"
    checkpointing: bool = False
    local: bool = True
    checkInterval: int = 5000
    stateBackend: str = "file:///tmp/omldm_checkpoints"
    trainingDataTopic: str = "trainingData"
    trainingDataAddr: str = "localhost:9092"
    forecastingDataTopic: str = "forecastingData"
    forecastingDataAddr: str = "localhost:9092"
    requestsTopic: str = "requests"
    requestsAddr: str = "localhost:9092"
    psMessagesTopic: str = "psMessages"
    psMessagesAddr: str = "localhost:9092"
    responsesTopic: str = "responses"
    responsesAddr: str = "localhost:9092"
    predictionsTopic: str = "predictions"
    predictionsAddr: str = "localhost:9092"
    performanceTopic: str = "performance"
    performanceAddr: str = "localhost:9092"
    test: bool = True
    maxMsgParams: int = 2000
    timeout: int = 30000
    testSetSize: int = 256
    # ---- reference constants made configurable
    recordBufferSize: int = 100000        # SpokeLogic.scala:32
    requestBufferSize: int = 10000        # SpokeLogic.scala:35
    queryBucketSize: int = 10000          # FlinkNetwork.scala:50
    bucketBytes: int = 64 << 20           # cap of one coalesced collective bucket
    seed: int = 25                        # FlinkSpoke.scala:52: default seed of seeded learners
    # ---- MI355X-native engine
    numFeatures: int = 13                 # numerical features per point (dense slots)
    discreteFeatures: int = 0             # discrete features per point (dense slots)
    catFeatures: int = 26                 # categorical features per point (hashed)
    hashDim: int = 1 << 20                # hashed feature space (incl. dense slots, intercept)
    fieldAware: bool = True               # compact uint16 field-aware slots (read by the v3 scan)
    batchSize: int = 65536                # records per engine tick and rank
    spokesPerDevice: int = 0              # virtual spokes per rank (0: parallelism / world)
    # Creates wait while the job runs below the spoke parallelism it has reached before
    # (a restore onto fewer spokes); FlinkSpoke.scala:69-71,145-156,345-348
    parallelismGate: bool = True
    device: str = "auto"                  # auto | cuda | cpu
    maxTicks: int = 0                     # 0: until terminated (tests use a bound)
    restore: bool = False                 # restore from the latest checkpoint in stateBackend
    checkpointExport: bool = True         # checkpoints also export models.json (Create requests)
    watchdogTimeout: int = 0              # ms without a finished tick → abort + exit (0: off)
    parseThreads: int = 8
    gpuParse: bool = True                 # parse + hash JSON records on the GPU (cuda only)
    prefetch: str = "auto"                # read tick k+1 while tick k trains (auto: on GPU)
    ingestCUs: int = 32                   # GPU: CUs (one XCD) for ingest copies; 0 off (profiles/round5/e2e_*.json)
    ingestCopy: str = "pull"              # GPU staging copy: pull (kernel) | sdma (hipMemcpyAsync)
    forecastServer: str = "auto"          # per-record forecasts on the resident serving wave (auto: GPU)
    pipelineStreams: int = 8              # GPU: pipelines of a tick train on up to this many streams
    fusePipelines: str = "true"           # GPU: hashed-linear pipelines sharing a prep: one launch
    routeAhead: str = "false"             # GPU: holdout route + v3 prep beside the previous round
    roundRows: int = 8192                 # rows per spoke per round: larger ticks run more rounds
    prepAhead: str = "true"               # GPU: later rounds' v3 preps beside the tick's first scan
    extra: dict = field(default_factory=dict)

    @staticmethod
    def from_args(argv=None) -> "JobConfig":
        """Flink ParameterTool style: ``--key value`` pairs; unknown keys land in ``extra``."""
        argv = list(argv or [])
        cfg = JobConfig()
        names = {f.name: f for f in fields(JobConfig) if f.name != "extra"}
        i = 0
        while i < len(argv):
            a = argv[i]
            if not a.startswith("-"):
                i += 1
                continue
            key = a.lstrip("-")
            val = "true"
            if "=" in key:
                key, val = key.split("=", 1)
            elif i + 1 < len(argv) and not argv[i + 1].startswith("--"):
                val = argv[i + 1]
                i += 1
            i += 1
            if key in names:
                typ = names[key].type
                if typ in ("bool", bool):
                    setattr(cfg, key, _bool(val))
                elif typ in ("int", int):
                    setattr(cfg, key, int(float(val)))
                else:
                    setattr(cfg, key, val)
            else:
                cfg.extra[key] = val
        return cfg

    def as_dict(self) -> dict:
        return asdict(self)


def argparser() -> argparse.ArgumentParser:
    """argparse mirror (for --help); parsing itself uses JobConfig.from_args."""
    ap = argparse.ArgumentParser(prog="omldm", description="MI355X-native online ML engine")
    for f in fields(JobConfig):
        if f.name == "extra":
            continue
        ap.add_argument(f"--{f.name}", default=getattr(JobConfig, f.name, None))
    return ap
