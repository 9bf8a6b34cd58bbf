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


def reduce_query_metrics(comm, answers: list, fitted: int, cum_loss: float,
                         mean_buffer: float = 0.0, spokes: int = 1) -> dict:
    """ResponseConstructor merge (omldm/utils/ResponseConstructor.scala:32-52) over every
    virtual spoke of every rank: each spoke answers from its own test set
    (FlinkSpoke.scala:160-163) with its mean loss and its score; dataFitted is summed,
    loss / score averaged over the answering spokes (all P once every test set holds a
    point), cumulativeLoss over all P spokes. ``answers``: this rank's (mean loss, score,
    test points) per spoke with test points; ``spokes``: this rank's spoke count, whose
    running totals (``fitted``, ``cum_loss``) the rank keeps jointly. ``meanBufferSize``:
    every spoke reports its mean buffer size / P and the statistics operator sums them
    (FlinkSpoke.scala:138, StatisticsOperator.scala:101) — the mean over spokes."""
    dev = "cpu"
    S = max(1, int(spokes))
    per = torch.tensor([sum(a[0] for a in answers), sum(a[1] for a in answers), float(fitted),
                        S * cum_loss / max(fitted, 1), float(sum(a[2] for a in answers)),
                        float(len(answers)), S * float(mean_buffer), float(S)],
                       dtype=torch.float64, device=dev)
    if comm.world > 1 and comm.backend == "nccl":
        per = per.to(torch.device("cuda", torch.cuda.current_device()))
    comm.all_reduce_(per, tag="query")
    per = per.cpu()
    workers = max(1.0, float(per[5]))
    P = max(1.0, float(per[7]))
    return {"loss": float(per[0]) / workers, "score": float(per[1]) / workers,
            "dataFitted": int(per[2]), "cumulativeLoss": float(per[3]) / P,
            "testPoints": int(per[4]), "workers": int(per[5]), "spokes": int(P),
            "meanBufferSize": float(per[6]) / P}


def split_params(params: dict | None, bucket: int = 10000) -> list[dict]:
    """FlinkNetwork.split (omldm/network/FlinkNetwork.scala:48-149): every value is cut
    into buckets of ``bucket`` elements — lists by element, strings by character — keyed
    ``name[start-end]``; bucket i collects the i-th slice of every parameter. A value
    that fits one bucket keeps its name; a one-element value or slice is unwrapped to
    the element (``params.head``); a scalar is a one-element value; an empty list or
    null yields no bucket."""
    if not params:
        return []
    buckets: dict[int, dict] = {}
    for name, val in params.items():
        if val is None:
            arr = []
        elif isinstance(val, (list, tuple, str)):
            arr = val
        else:
            arr = [val]
        n = len(arr)
        nb = n // bucket + (0 if n % bucket == 0 else 1)
        if nb == 1:
            buckets.setdefault(0, {})[name] = arr[0] if n == 1 else (
                arr if isinstance(arr, str) else list(arr))
            continue
        for i in range(nb):
            s = i * bucket
            e = (s + n % bucket - 1) if (i == nb - 1 and n % bucket) else (i + 1) * bucket - 1
            sl = arr[s:e + 1]
            buckets.setdefault(i, {})[f"{name}[{s}-{e}]"] = sl[0] if len(sl) == 1 else (
                sl if isinstance(sl, str) else list(sl))
    return [buckets[i] for i in sorted(buckets)]


_BUCKET_KEY = None


def merge_bucketed(params: dict | None) -> dict:
    """Inverse of ``split_params`` over the union of a response's bucket maps: keys
    ``name[start-end]`` are reassembled into ``name`` (lists concatenated in start order,
    strings joined); other keys pass through. What a user does to re-create a pipeline
    from a bucketed QueryResponse (Create with ``learner.parameters``)."""
    import re

    global _BUCKET_KEY
    if _BUCKET_KEY is None:
        _BUCKET_KEY = re.compile(r"^(.*)\[(\d+)-(\d+)\]$")
    if not params:
        return {}
    parts: dict[str, list] = {}
    out: dict = {}
    for k, v in params.items():
        m = _BUCKET_KEY.match(k)
        if m is None:
            out[k] = v
            continue
        parts.setdefault(m.group(1), []).append((int(m.group(2)), int(m.group(3)), v))
    for name, segs in parts.items():
        segs.sort()
        if all(isinstance(v, str) for _, _, v in segs):
            out[name] = "".join(v for _, _, v in segs)
            continue
        flat: list = []
        for s, e, v in segs:
            if len(flat) != s:
                raise ValueError(f"bucketed parameter {name!r}: gap before [{s}-{e}]")
            flat.extend(v if isinstance(v, list) else [v])
        out[name] = flat
    return out


def build_query_responses(response_id: int, mlp_id: int, preprocessors: list, learner: dict,
                          protocol: str, metrics: dict, bucket: int = 10000) -> list[QueryResponse]:
    """The reference's sendQueryResponse (FlinkNetwork.scala:151-240): with at most two
    buckets of parameters / hyper-parameters / data structure the response goes out
    whole (``maxBuckets < 2``); otherwise one response per bucket index, the statistics
    fields (preprocessors, protocol, dataFitted, loss, cumulativeLoss, score) riding on
    the last parameter bucket (the last bucket when there are no parameters — the
    reference drops them in that case)."""
    pb = split_params(learner.get("parameters"), bucket)
    hb = split_params(learner.get("hyperParameters"), bucket)
    sb = split_params(learner.get("dataStructure"), bucket)
    nb = max(len(pb), len(hb), len(sb), 1)
    if nb - 1 < 2:
        return [QueryResponse(response_id, 0, mlp_id, preprocessors, learner, protocol,
                              metrics["dataFitted"], metrics["loss"], metrics["cumulativeLoss"],
                              metrics["score"])]
    stats_at = len(pb) - 1 if pb else nb - 1
    out = []
    for i in range(nb):
        part = {"name": learner.get("name"),
                "parameters": pb[i] if i < len(pb) else None,
                "hyperParameters": hb[i] if i < len(hb) else None,
                "dataStructure": sb[i] if i < len(sb) else None}
        st = i == stats_at
        out.append(QueryResponse(response_id, i, mlp_id, preprocessors if st else None, part,
                                 protocol if st else None,
                                 metrics["dataFitted"] if st else None,
                                 metrics["loss"] if st else None,
                                 metrics["cumulativeLoss"] if st else None,
                                 metrics["score"] if st else None))
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


def merge_hub_statistics(hub_stats: list[dict], fitted: int) -> dict:
    """StatisticsAggregateFunction.getResult (StateAccumulators.scala:94-108): the records
    of a pipeline's H hubs are summed (updateStats), then blocks, models and fitted are
    divided by H — bytes stay summed."""
    H = max(1, len(hub_stats))
    tot = {k: sum(int(h[k]) for h in hub_stats) for k in
           ("modelsShipped", "bytesShipped", "numOfBlocks")}
    return {"modelsShipped": tot["modelsShipped"] // H, "bytesShipped": tot["bytesShipped"],
            # every hub counts the pipeline's global fitted examples: H·fitted / H
            "numOfBlocks": tot["numOfBlocks"] // H, "fitted": fitted, "hubs": H}


def pipeline_statistics(pipe, metrics: dict | None = None) -> Statistics:
    ps = pipe.protocol.stats
    pipe.flush_learning_curve()
    lc = pipe.learning_curve
    fitted = int(metrics["dataFitted"]) if metrics else pipe.learner.running_totals()["fitted"]
    merged = merge_hub_statistics(pipe.protocol.hub_statistics(), fitted)
    st = Statistics(pipeline=pipe.id, protocol=pipe.protocol_name,
                    modelsShipped=merged["modelsShipped"], bytesShipped=merged["bytesShipped"],
                    numOfBlocks=merged["numOfBlocks"], fitted=merged["fitted"],
                    learningCurve=[x[0] for x in lc] or None, lcx=[x[1] for x in lc] or None,
                    meanBufferSize=float(metrics.get("meanBufferSize", 0.0)) if metrics else
                    pipe.mean_buffer_size(),
                    score=metrics["score"] if metrics else None,
                    extra={"syncs": ps.syncs, "rounds": ps.rounds, "hubs": merged["hubs"],
                           "smallMessages": ps.small_messages})
    return st


def job_statistics(job_name: str, parallelism: int, duration_ms: int, stats: list) -> JobStatistics:
    """``parallelism`` is the job's spoke parallelism (StatisticsOperator.scala:109-113:
    the operator's parallelism = the spoke count P), i.e. spokes per rank × ranks."""
    return JobStatistics(job_name, parallelism, duration_ms, sorted(stats, key=lambda s: s.pipeline))
