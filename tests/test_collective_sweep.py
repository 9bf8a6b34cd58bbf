"""bench/collective_sweep.py (SURVEY §5.8 bucket sizing) on 2 gloo ranks: every sweep
emits its JSON lines and the coalesced/bucketed paths finish."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_collective_sweep_two_ranks():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench", "collective_sweep.py"), "--sizes", "4096,65536",
           "--iters", "2", "--warmup", "1", "--pipelines", "3", "--dim-log2", "12",
           "--caps", "16384,1048576", "--parts", "1,3"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-2000:]
    recs = [json.loads(l) for l in out.stdout.splitlines() if l.startswith("{")]
    kinds = {r["sweep"] for r in recs}
    assert kinds == {"op", "bucket", "parts"}
    assert all(r["world"] == 2 and r["us"] > 0 for r in recs)
    ops = {r["op"] for r in recs if r["sweep"] == "op"}
    assert {"all_reduce (H=G)", "reduce+bcast (H=1)", "reduce_scatter", "all_gather"} <= ops
