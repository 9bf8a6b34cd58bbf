"""Job statistics, query-response reduction and idle termination.

Reference:
* hub-side ``Statistics`` per message in test mode (protocol, modelsShipped, bytesShipped,
  numOfBlocks, fitted, learning-curve slices from hub 0) — omldm/operators/hub/
  FlinkHub.scala:88-157; merged per pipeline (omldm/state/StateAccumulators.scala:54-126);
* StatisticsOperator: start = first statistic, end = latest; an idle timer of ``timeout``
  ms emits the termination signal; after every worker answered the −1 query it emits
  ``JobStatistics(jobName, P, end − start, stats)`` with the normalised score
  (omldm/utils/statistics/StatisticsOperator.scala:69-142);
* ResponseConstructor: gathers the P worker responses of a query, sums ``dataFitted`` and
  averages loss / cumulativeLoss / score (omldm/utils/ResponseConstructor.scala:17-61);
* query responses are split into buckets of 10,000 parameters keyed ``name[start-end]``
  (omldm/network/FlinkNetwork.scala:48-149).
Here the P-way gather is one all-reduce of a small vector; the idle detector runs on
wall-clock time (the reference's event-time timer never fires without watermarks —
SURVEY §2.8 Q7).
"""
from __future__ import annotations

import time

import torch

from omldm_amd.api.schemas import JobStatistics, QueryResponse, Statistics


def reduce_query_metrics(comm, loss_sum: float, score_sum: float, n: int, fitted: int,
                         cum_loss: float) -> dict:
    """ResponseConstructor merge over ranks: Σ fitted; loss/cumLoss/score averaged over
    workers of per-worker means (reference semantics)."""
    dev = "cpu"
    per = torch.tensor([loss_sum / max(n, 1), score_sum / max(n, 1), float(fitted),
                        cum_loss / max(fitted, 1), float(n), 1.0 if n > 0 else 0.0],
                       dtype=torch.float64, device=dev)
    if comm.world > 1 and comm.backend == "nccl":
        per = per.to(torch.device("cuda", torch.cuda.current_device()))
    comm.all_reduce_(per, tag="query")
    per = per.cpu()
    workers = max(1.0, float(per[5]))
    return {"loss": float(per[0]) / workers, "score": float(per[1]) / workers,
            "dataFitted": int(per[2]), "cumulativeLoss": float(per[3]) / workers,
            "testPoints": int(per[4]), "workers": int(workers)}


def split_params(params: dict | None, bucket: int = 10000) -> list[dict]:
    """FlinkNetwork.split: every list longer than ``bucket`` is cut into buckets keyed
    ``name[start-end]``; bucket i collects the i-th slice of every parameter."""
    if not params:
        return []
    buckets: dict[int, dict] = {}
    for name, val in params.items():
        arr = val if isinstance(val, (list, tuple)) else [val]
        n = len(arr)
        nb = n // bucket + (0 if n % bucket == 0 else 1)
        if nb <= 1:
            buckets.setdefault(0, {})[name] = arr[0] if n == 1 and not isinstance(val, list) \
                else val
            continue
        for i in range(nb):
            s = i * bucket
            e = min(n, s + bucket) - 1
            buckets.setdefault(i, {})[f"{name}[{s}-{e}]"] = list(arr[s:e + 1])
    return [buckets[i] for i in sorted(buckets)]


def build_query_responses(response_id: int, mlp_id: int, preprocessors: list, learner: dict,
                          protocol: str, metrics: dict, bucket: int = 10000) -> list[QueryResponse]:
    """One QueryResponse, or bucketed ones when the parameters exceed one bucket; the
    statistics fields ride on the last bucket (FlinkNetwork.scala:187-237)."""
    pb = split_params(learner.get("parameters"), bucket)
    hb = split_params(learner.get("hyperParameters"), bucket)
    sb = split_params(learner.get("dataStructure"), bucket)
    nb = max(len(pb), len(hb), len(sb), 1)
    if nb < 2:
        return [QueryResponse(response_id, 0, mlp_id, preprocessors, learner, protocol,
                              metrics["dataFitted"], metrics["loss"], metrics["cumulativeLoss"],
                              metrics["score"])]
    out = []
    for i in range(nb):
        part = {"name": learner.get("name"),
                "parameters": pb[i] if i < len(pb) else None,
                "hyperParameters": hb[i] if i < len(hb) else None,
                "dataStructure": sb[i] if i < len(sb) else None}
        last = i == nb - 1
        out.append(QueryResponse(response_id, i, mlp_id, preprocessors if last else None, part,
                                 protocol if last else None,
                                 metrics["dataFitted"] if last else None,
                                 metrics["loss"] if last else None,
                                 metrics["cumulativeLoss"] if last else None,
                                 metrics["score"] if last else None))
    return out


class IdleDetector:
    """Wall-clock idle timeout (reference: event-time timer ts + timeout)."""

    def __init__(self, timeout_ms: int):
        self.timeout = timeout_ms / 1000.0
        self.start = None
        self.last = time.time()
        self.end = None

    def activity(self, now: float | None = None):
        now = now or time.time()
        if self.start is None:
            self.start = now
        self.last = now
        self.end = now

    def expired(self, now: float | None = None) -> bool:
        now = now or time.time()
        return self.start is not None and now - self.last >= self.timeout

    def duration_ms(self) -> int:
        if self.start is None:
            return 0
        return int(((self.end or self.start) - self.start) * 1000)


def pipeline_statistics(pipe, metrics: dict | None = None) -> Statistics:
    ps = pipe.protocol.stats
    lc = pipe.learning_curve
    st = Statistics(pipeline=pipe.id, protocol=pipe.protocol_name,
                    modelsShipped=ps.models_shipped, bytesShipped=ps.bytes_shipped,
                    numOfBlocks=ps.num_of_blocks,
                    fitted=int(metrics["dataFitted"]) if metrics else
                    pipe.learner.running_totals()["fitted"],
                    learningCurve=[x[0] for x in lc] or None, lcx=[x[1] for x in lc] or None,
                    score=metrics["score"] if metrics else None,
                    extra={"syncs": ps.syncs, "rounds": ps.rounds,
                           "smallMessages": ps.small_messages})
    return st


def job_statistics(job_name: str, parallelism: int, duration_ms: int, stats: list) -> JobStatistics:
    return JobStatistics(job_name, parallelism, duration_ms, sorted(stats, key=lambda s: s.pipeline))
