"""User-facing JSON payloads: Request, DataInstance, QueryResponse, Prediction,
Statistics, JobStatistics — field names kept compatible with the reference's ControlAPI
POJOs as used by OMLDM:

* Request:       omldm/utils/parsers/requestStream/PipelineMap.scala:22-45,
                 omldm/operators/spoke/FlinkSpoke.scala:142-184
* DataInstance:  omldm/utils/parsers/dataStream/DataPointParser.scala:17-46
* QueryResponse: omldm/network/FlinkNetwork.scala:196-230 (10-field ctor),
                 omldm/utils/ResponseConstructor.scala:33-53
* Statistics:    omldm/operators/hub/FlinkHub.scala:118-153 (8-field ctor),
                 omldm/state/StateAccumulators.scala:54-126
* JobStatistics: omldm/utils/statistics/StatisticsOperator.scala:111-126
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field
from typing import Any

REQUEST_TYPES = ("Create", "Update", "Query", "Delete")
VALID_LEARNERS = ("PA", "RegressorPA", "ORR", "SVM", "MultiClassPA", "K-means", "NN", "HT")
VALID_PREPROCESSORS = ("PolynomialFeatures", "StandardScaler", "MinMaxScaler")
# Extensions beyond the reference's list (BASELINE.json config 2) — accepted as well.
EXTENSION_LEARNERS = ("LogisticRegression",)
SINGLE_LEARNER_MODELS = ("HT", "K-means")


def _clean(d: dict) -> dict:
    return {k: v for k, v in d.items() if v is not None}


@dataclass
class LearnerPOJO:
    name: str | None = None
    hyperParameters: dict | None = None
    parameters: dict | None = None
    dataStructure: dict | None = None

    @staticmethod
    def from_obj(o) -> "LearnerPOJO | None":
        if o is None:
            return None
        if isinstance(o, LearnerPOJO):
            return o
        return LearnerPOJO(o.get("name"), o.get("hyperParameters") or o.get("hyperparameters"),
                           o.get("parameters"), o.get("dataStructure"))

    def to_obj(self) -> dict:
        return _clean(asdict(self))


@dataclass
class PreprocessorPOJO:
    name: str | None = None
    hyperParameters: dict | None = None
    parameters: dict | None = None
    dataStructure: dict | None = None

    @staticmethod
    def from_obj(o) -> "PreprocessorPOJO":
        if isinstance(o, PreprocessorPOJO):
            return o
        return PreprocessorPOJO(o.get("name"), o.get("hyperParameters") or o.get("hyperparameters"),
                                o.get("parameters"), o.get("dataStructure"))

    def to_obj(self) -> dict:
        return _clean(asdict(self))


@dataclass
class Request:
    id: int | None = None
    request: str | None = None
    requestId: int | None = None
    learner: LearnerPOJO | None = None
    preProcessors: list[PreprocessorPOJO] | None = None
    trainingConfiguration: dict = field(default_factory=dict)

    @staticmethod
    def from_json(s: str | bytes | dict) -> "Request":
        o = json.loads(s) if isinstance(s, (str, bytes, bytearray)) else dict(s)
        pps = o.get("preProcessors") or o.get("preprocessors")
        rid = o.get("requestId")
        return Request(
            id=o.get("id"),
            request=o.get("request"),
            requestId=int(rid) if rid is not None else None,
            learner=LearnerPOJO.from_obj(o.get("learner")),
            preProcessors=[PreprocessorPOJO.from_obj(p) for p in pps] if pps else None,
            trainingConfiguration=dict(o.get("trainingConfiguration") or {}),
        )

    def is_valid(self) -> bool:
        if not isinstance(self.id, int) or isinstance(self.id, bool) or self.id < 0:
            return False
        if self.request not in REQUEST_TYPES:
            return False
        if self.request == "Create" and (self.learner is None or not self.learner.name):
            return False
        return True

    def to_obj(self) -> dict:
        return _clean({
            "id": self.id, "request": self.request, "requestId": self.requestId,
            "learner": self.learner.to_obj() if self.learner else None,
            "preProcessors": [p.to_obj() for p in self.preProcessors] if self.preProcessors else None,
            "trainingConfiguration": self.trainingConfiguration or None,
        })

    def to_json(self) -> str:
        return json.dumps(self.to_obj())


@dataclass
class DataInstance:
    numericalFeatures: list | None = None
    discreteFeatures: list | None = None
    categoricalFeatures: list | None = None
    target: float | None = None
    operation: str = "training"
    id: Any = None

    @staticmethod
    def from_json(s) -> "DataInstance":
        o = json.loads(s) if isinstance(s, (str, bytes, bytearray)) else dict(s)
        return DataInstance(o.get("numericalFeatures"), o.get("discreteFeatures"),
                            o.get("categoricalFeatures"), o.get("target"),
                            o.get("operation", "training"), o.get("id"))

    def is_valid(self) -> bool:
        if self.numericalFeatures is None and self.discreteFeatures is None and \
                self.categoricalFeatures is None:
            return False
        if self.operation not in ("training", "forecasting"):
            return False
        return not (self.operation == "training" and self.target is None)

    def to_json(self) -> str:
        return json.dumps(_clean(asdict(self)))


@dataclass
class QueryResponse:
    responseId: int
    id: int = 0                       # bucket index (FlinkNetwork.scala:196-230)
    mlpId: int | None = None
    preprocessors: list | None = None
    learner: dict | None = None
    protocol: str | None = None
    dataFitted: int | None = None
    loss: float | None = None
    cumulativeLoss: float | None = None
    score: float | None = None

    def to_obj(self) -> dict:
        return _clean(asdict(self))

    def to_json(self) -> str:
        return json.dumps(self.to_obj())

    @staticmethod
    def from_json(s) -> "QueryResponse":
        o = json.loads(s) if isinstance(s, (str, bytes, bytearray)) else dict(s)
        return QueryResponse(**{k: o.get(k) for k in QueryResponse.__dataclass_fields__})


@dataclass
class Prediction:
    mlpId: int
    dataPoint: Any
    prediction: float

    def to_json(self) -> str:
        dp = self.dataPoint
        if isinstance(dp, (bytes, bytearray)):
            dp = dp.decode()
        if isinstance(dp, str):
            try:
                dp = json.loads(dp)
            except ValueError:
                pass
        return json.dumps({"mlpId": self.mlpId, "dataPoint": dp, "prediction": self.prediction})


@dataclass
class Statistics:
    pipeline: int
    protocol: str | None = None
    modelsShipped: int = 0
    bytesShipped: int = 0
    numOfBlocks: int = 0
    fitted: int = 0
    learningCurve: list | None = None
    lcx: list | None = None
    meanBufferSize: float = 0.0
    score: float | None = None
    extra: dict | None = None

    def to_obj(self) -> dict:
        return _clean(asdict(self))


@dataclass
class JobStatistics:
    jobName: str
    parallelism: int
    duration: int                      # ms between the first and last statistic
    statistics: list[Statistics] = field(default_factory=list)
    metrics: dict | None = None        # engine metrics (extension)

    def to_json(self) -> str:
        o = {"jobName": self.jobName, "parallelism": self.parallelism,
             "duration": self.duration, "statistics": [s.to_obj() for s in self.statistics]}
        if self.metrics is not None:
            o["metrics"] = self.metrics
        return json.dumps(o)
