"""Command line entry point: ``python -m omldm_amd --flag value ...`` (one process per GPU;
multi-GPU: ``python -m torch.distributed.run --nproc-per-node N -m omldm_amd ...``).

Reference: ``flink run ... omldm.Job --parallelism 16 --trainingDataAddr ...``
(README.md:28-41, omldm/Job.scala:110-168); the same flag names are accepted
(omldm_amd/utils/config.py).
"""
from __future__ import annotations

import json
import sys

from omldm_amd.utils.config import JobConfig, argparser


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if "-h" in argv or "--help" in argv:
        argparser().print_help()
        return 0
    cfg = JobConfig.from_args(argv)
    from omldm_amd.engine.job import Job
    from omldm_amd.parallel.comm import init_distributed

    comm, device = init_distributed(cfg.device)
    job = Job(cfg, comm, device).run()
    if comm.rank == 0:
        print(json.dumps({"job": cfg.jobName, "ticks": job.ticks, "counters": job.counters,
                          "terminated": job.terminated}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
