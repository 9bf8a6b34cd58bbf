"""A rank-local engine inside a multi-rank job never issues a collective: the bench's
rank-0 side measurements (engine forecast latency, engine end-to-end rate) run a Job on
``Comm.local()`` while the other ranks wait at the final barrier (bench.py)."""
import json
import os
import socket
import tempfile
import uuid

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.engine.job import Job
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import MemoryBroker
from omldm_amd.parallel.comm import Comm
from omldm_amd.utils.config import JobConfig


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fitted = 0
    if rank == 0:
        name = uuid.uuid4().hex
        args = []
        for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
                  "predictionsAddr", "performanceAddr"):
            args += [f"--{k}", f"memory://{name}"]
        cfg = JobConfig.from_args(args + ["--hashDim", str(1 << 14), "--batchSize", "500",
                                          "--timeout", "100", "--test", "false"])
        br = MemoryBroker.named(name)
        br.produce("requests", json.dumps({"id": 1, "request": "Create",
                                           "learner": {"name": "SVM"},
                                           "trainingConfiguration": {"protocol": "Synchronous"}}))
        for r in synth_json_records(2000, FeatureSpace(13, 0, 26, 1 << 14)):
            br.produce("trainingData", r)
        comm = Comm.local()
        assert comm.world == 1 and comm.rank == 0
        job = Job(cfg, comm, "cpu")
        for _ in range(6):
            job.tick()
        fitted = job.pipes[1].learner.running_totals()["fitted"]
        assert comm.stats.collectives == 0 or all(
            k == "host_all_reduce" for k, _, _ in (comm.stats.trace or []))
    dist.barrier()
    torch.save({"fitted": fitted}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_rank_local_job_inside_a_two_rank_job():
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _port(), d), nprocs=2, start_method="fork")
        res = [torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True) for r in range(2)]
    assert res[0]["fitted"] > 0
