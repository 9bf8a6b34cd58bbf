"""The examples keep working (CPU)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_quickstart_runs_on_cpu():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "quickstart.py"), "--cpu",
                          "--records", "6000"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "prediction:" in out.stdout and "performance:" in out.stdout
    assert "response 100" in out.stdout and "response 200" in out.stdout
