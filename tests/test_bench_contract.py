"""bench.py driver contract on the CPU (gloo): one JSON line from rank 0 with the fields
the driver reads, for 1 rank and for 2 ranks under torch.distributed.run (max over
ranks, whole-job value, reduce-slice tuning at N > 1), and the config-2 learner."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "2", "--warmup", "1", "--spokes", "4", "--rows", "64", "--pool", "2",
         "--latency-samples", "3", "--dim-log2", "16"]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _run(cmd):
    env = dict(os.environ, OMP_NUM_THREADS="1", OMLDM_CPU_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-3000:]
    return _json_lines(out.stdout)


def test_bench_one_rank_contract():
    recs = _run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL])
    assert len(recs) == 1
    r = recs[0]
    assert KEYS <= set(r)
    assert r["n_gpus"] == 1 and r["steps"] == 2 and r["warmup"] == 1
    assert r["higher_is_better"] is True and r["scaling"] == "weak" and r["value"] > 0
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(r["config"])
    assert r["config"]["global_batch"] == 4 * 64 and r["config"]["parallelism"] == "dp1"
    assert "B/example" in r["data"] and "synthetic" in r["data"] and "tokens" in r["data"]
    # quality next to speed: the same stream through the CPU reference semantics
    assert r["dtype"] == "fp32" and r["ref_holdout_accuracy"] is not None
    assert abs(r["accuracy_gap_pt"]) <= 0.5


def test_bench_logistic_regression_config2():
    recs = _run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL,
                 "--learner", "LogisticRegression"])
    assert "logistic regression" in recs[0]["metric"]
    assert recs[0]["config"]["model"].startswith("logistic regression")


def test_bench_two_ranks_contract():
    recs = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                 "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                 str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", *SMALL])
    assert len(recs) == 1  # rank 0 only
    r = recs[0]
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2"
    assert r["config"]["global_batch"] == 2 * 4 * 64
    assert r["backend"] == "gloo" and abs(r["accuracy_gap_pt"]) <= 0.5


def test_bench_eight_ranks_rehearsal():
    """The driver's N=8 scaling run, rehearsed on gloo: 8 ranks under torch.distributed.run,
    rank 0 alone prints the whole-job line (MAX of the ranks' times)."""
    recs = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                 "--nproc-per-node", "8", "--master-addr", "127.0.0.1", "--master-port",
                 str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "8", *SMALL])
    assert len(recs) == 1
    r = recs[0]
    assert r["n_gpus"] == 8 and r["config"]["parallelism"] == "dp8"
    assert r["config"]["global_batch"] == 8 * 4 * 64
    assert r["value"] > 0 and r["ref_semantics"].startswith("CPU sequential PA-I, P=32")
