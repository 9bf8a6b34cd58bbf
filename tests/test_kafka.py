"""Kafka transport: RecordBatch v2 codec, CRC-32C, client ↔ protocol-level fake broker,
and a whole engine job driven through Kafka topics."""
import json
import uuid

from omldm_amd.io.kafka import KafkaBroker, crc32c, decode_batches, encode_batch, read_varint, \
    varint
from omldm_amd.io.transport import Consumer
from tests.fake_kafka import FakeKafka


def test_crc32c_known_vector():
    assert crc32c(b"123456789") == 0xE3069283
    assert crc32c(b"") == 0


def test_varint_roundtrip():
    for v in (0, 1, -1, 63, -64, 300, -300, 2**31, -(2**31)):
        b = varint(v)
        assert read_varint(b, 0) == (v, len(b))


def test_record_batch_roundtrip():
    vals = [json.dumps({"i": i}).encode() for i in range(50)]
    data = encode_batch(vals, base_offset=100) + encode_batch([b"x"], base_offset=150)
    got = decode_batches(data)
    assert [o for o, _ in got] == list(range(100, 151))
    assert [v for _, v in got][:50] == vals
    assert decode_batches(data[:-3]) == got[:50]  # truncated trailing batch ignored


def test_client_against_fake_broker():
    fk = FakeKafka(default_partitions=4)
    try:
        br = KafkaBroker(fk.addr)
        br.create_topic("trainingData", 4)
        assert br.partitions("trainingData") == 4
        for i in range(40):
            br.produce("trainingData", json.dumps({"i": i}))
        c0 = Consumer(br, "trainingData", rank=0, world=2)
        c1 = Consumer(br, "trainingData", rank=1, world=2)
        got = c0.poll(100) + c1.poll(100)
        assert sorted(json.loads(x)["i"] for x in got) == list(range(40))
        assert br.end_offset("trainingData", 0) == 10
        late = Consumer(br, "trainingData", start="latest", all_partitions=True)
        br.produce("trainingData", "tail", partition=2)
        assert late.poll(10) == [b"tail"]
        br.close()
    finally:
        fk.close()


def test_engine_over_kafka():
    from omldm_amd.api.batch import FeatureSpace
    from omldm_amd.engine.job import Job
    from omldm_amd.io.synthetic import synth_json_records
    from omldm_amd.parallel.comm import Comm
    from omldm_amd.utils.config import JobConfig

    fk = FakeKafka(default_partitions=2)
    try:
        args = []
        for k in ("trainingDataAddr", "forecastingDataAddr", "requestsAddr", "responsesAddr",
                  "predictionsAddr", "performanceAddr"):
            args += [f"--{k}", fk.addr]
        sp = FeatureSpace(13, 0, 26, 1 << 14)
        cfg = JobConfig.from_args(args + ["--hashDim", str(sp.dim), "--timeout", "300",
                                          "--batchSize", "400", "--jobName", uuid.uuid4().hex])
        br = KafkaBroker(fk.addr)
        for r in synth_json_records(600, sp):
            br.produce("trainingData", r)
        br.produce("requests", json.dumps({"id": 1, "request": "Create",
                                           "learner": {"name": "PA"},
                                           "trainingConfiguration": {"protocol": "Synchronous"}}))
        for r in synth_json_records(5, sp, start=7, operation="forecasting"):
            br.produce("forecastingData", r)
        job = Job(cfg, Comm(), "cpu").run()
        assert job.terminated and job.counters["predictions"] == 5
        perf = Consumer(br, "performance", all_partitions=True).poll(10)
        assert json.loads(perf[-1])["jobName"] == cfg.jobName
        preds = Consumer(br, "predictions", all_partitions=True).poll(100)
        assert len(preds) == 5
    finally:
        fk.close()
