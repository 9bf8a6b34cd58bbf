"""Request validation and routing (the control plane's single writer, rank 0).

Reference: PipelineMap (omldm/utils/parsers/requestStream/PipelineMap.scala:14-71), run
at parallelism 1 and keyed by 0 (omldm/Job.scala:149-153):
  * drop requests naming a learner/preprocessor outside the valid lists (:22-30, :66-69);
  * Create for a NEW id → remember it and broadcast to every worker (:31-34);
  * Update / Delete for a known id → broadcast (:35-36, :43-46);
  * Query for a known id → worker 0 only for HT and K-means, else broadcast (:37-42).
Malformed JSON is dropped and counted instead of killing the job.
"""
from __future__ import annotations

from dataclasses import dataclass

from omldm_amd.api.schemas import (EXTENSION_LEARNERS, SINGLE_LEARNER_MODELS, VALID_LEARNERS,
                                   VALID_PREPROCESSORS, Request)

ALL = -1  # destination: every worker


@dataclass
class ControlMessage:
    """Reference ControlMessage(networkId, operation, source, destination, data, request)
    (omldm/messages/ControlMessage.scala:18-74); here destination ALL == broadcast."""

    network_id: int
    destination: int
    request: Request


class PipelineMap:
    def __init__(self, allow_extensions: bool = True):
        self.node_map: dict[int, Request] = {}
        self.allow_extensions = allow_extensions
        self.dropped = 0

    def learner_ok(self, name: str | None) -> bool:
        return name in VALID_LEARNERS or (self.allow_extensions and name in EXTENSION_LEARNERS)

    def process(self, request: Request | str | bytes | dict) -> list[ControlMessage]:
        try:
            req = request if isinstance(request, Request) else Request.from_json(request)
        except (ValueError, TypeError, AttributeError):
            self.dropped += 1
            return []
        if not req.is_valid():
            self.dropped += 1
            return []
        if req.learner is not None and req.learner.name is not None and \
                not self.learner_ok(req.learner.name):
            self.dropped += 1
            return []
        if req.preProcessors and not all(p.name in VALID_PREPROCESSORS for p in req.preProcessors):
            self.dropped += 1
            return []
        rid = req.id
        if req.request == "Create":
            if rid in self.node_map:
                self.dropped += 1
                return []
            self.node_map[rid] = req
            return [ControlMessage(rid, ALL, req)]
        if rid not in self.node_map:
            self.dropped += 1
            return []
        if req.request == "Update":
            return [ControlMessage(rid, ALL, req)]
        if req.request == "Query":
            if self.node_map[rid].learner.name in SINGLE_LEARNER_MODELS:
                return [ControlMessage(rid, 0, req)]
            return [ControlMessage(rid, ALL, req)]
        if req.request == "Delete":
            del self.node_map[rid]
            return [ControlMessage(rid, ALL, req)]
        return []

    def state_dict(self) -> dict:
        return {"node_map": {k: v.to_obj() for k, v in self.node_map.items()},
                "dropped": self.dropped}

    def load_state_dict(self, sd: dict) -> None:
        self.node_map = {int(k): Request.from_json(v) for k, v in sd.get("node_map", {}).items()}
        self.dropped = sd.get("dropped", 0)
