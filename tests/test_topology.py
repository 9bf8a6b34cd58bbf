"""NUMA placement helpers (omldm_amd/utils/topology.py) against a fake sysfs tree."""
import os

from omldm_amd.utils import topology as T


def test_parse_cpulist():
    assert T.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert T.parse_cpulist("") == []


def test_device_locality_fake_sysfs(tmp_path):
    d = tmp_path / "0000:26:00.0"
    d.mkdir()
    (d / "numa_node").write_text("1\n")
    (d / "local_cpulist").write_text("64-67,192\n")
    node, cpus = T.device_locality("0000:26:00.0", str(tmp_path))
    assert node == 1 and cpus == [64, 65, 66, 67, 192]
    assert T.device_locality("0000:99:00.0", str(tmp_path)) is None


def test_bind_is_noop_without_gpu(monkeypatch):
    monkeypatch.setenv("OMLDM_NUMA_BIND", "1")
    before = os.sched_getaffinity(0)
    info = T.bind_to_device(0)
    assert info["numa_node"] is None
    assert os.sched_getaffinity(0) == before
