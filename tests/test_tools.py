"""Operator tools (python -m omldm_amd.tools) against file topics and the Kafka fake broker."""
import json

import pytest

from omldm_amd import tools
from omldm_amd.io.transport import Consumer, broker_for


def _flow(bootstrap, tmp_path, capsys):
    assert tools.main(["topics", "--bootstrap", bootstrap, "--data-partitions", "3"]) == 0
    assert tools.main(["synth", "--bootstrap", bootstrap, "--n", "3000", "--hash-dim",
                       str(1 << 14)]) == 0
    reqs = tmp_path / "r.jsonl"
    reqs.write_text("\n".join(json.dumps({"id": i, "request": "Query", "requestId": i})
                              for i in range(5)) + "\n")
    assert tools.main(["produce", "--bootstrap", bootstrap, "--topic", "requests",
                       "--file", str(reqs)]) == 0
    capsys.readouterr()
    assert tools.main(["tail", "--bootstrap", bootstrap, "--topic", "requests", "-n", "2"]) == 0
    lines = capsys.readouterr().out.strip().splitlines()
    assert [json.loads(x)["id"] for x in lines] == [3, 4]  # the last two, in order
    br = broker_for(bootstrap)
    counts = []
    for p in range(br.partitions("trainingData")):
        c = Consumer(br, "trainingData", all_partitions=True)
        c.parts = [p]
        n = 0
        while True:
            got = c.poll(10**6)
            if not got:
                break
            n += len(got)
        counts.append(n)
    assert sum(counts) == 3000 and max(counts) - min(counts) <= 1  # spread round-robin


def test_tools_on_file_topics(tmp_path, capsys):
    _flow(f"file://{tmp_path / 'topics'}", tmp_path, capsys)


def test_tools_on_kafka(tmp_path, capsys):
    from tests.fake_kafka import FakeKafka

    fk = FakeKafka(default_partitions=3)
    try:
        _flow(fk.addr, tmp_path, capsys)
    finally:
        fk.close()
