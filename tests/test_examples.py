"""The examples keep working (CPU)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_quickstart_runs_on_cpu():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "quickstart.py"), "--cpu",
                          "--records", "6000"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "prediction:" in out.stdout and "performance:" in out.stdout
    assert "response 100" in out.stdout and "response 200" in out.stdout


def test_single_node_recipe_two_ranks(tmp_path):
    """examples/single_node.sh end to end on two CPU ranks (torchrun, gloo): topics, data,
    requests, the job until its idle timeout, the answers read back."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, TOPICS=str(tmp_path / "topics"), NGPU="2", N="20000", PORT=str(port),
               OMP_NUM_THREADS="1")
    out = subprocess.run(["bash", os.path.join(ROOT, "examples", "single_node.sh")], cwd=ROOT,
                         env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-3000:])
    perf = [line for line in out.stdout.splitlines() if line.startswith('{"jobName"')]
    assert perf and '"parallelism": 2' in perf[-1]


@pytest.mark.gpu
def test_quickstart_runs_on_gpu(cuda):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "quickstart.py"),
                          "--records", "20000"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "response 100" in out.stdout and "performance:" in out.stdout
