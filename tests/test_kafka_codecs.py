"""Kafka compression codecs and the native record-set decoder (csrc/host/kafka_wire.cpp).

Each codec is checked against frames built by hand from its public format description
(so the decoders are not only tested against their own encoders): a raw and an
xerial-framed snappy stream, an LZ4 frame with an uncompressed block (header checksum by
the independent ``xxhash`` package), a zstd frame with a raw block, and gzip against
Python's ``gzip`` module in both directions. Then RecordBatch v2 with every codec through
the Python decoder and the native one, and the client against the fake broker (including
the Fetch v10 fallback that zstd topics need and transactional control batches).
"""
import gzip
import json
import os
import struct

import numpy as np
import pytest

from omldm_amd.io import kafka as K
from omldm_amd.io.transport import Consumer
from tests.fake_kafka import FakeKafka

CODECS = ["gzip", "snappy", "lz4", "zstd"]


def _need(codec):
    """lz4 / zstd come from the system's liblz4 / libzstd (loaded at run time)."""
    if codec not in ("none", None) and not K.codec_available(codec):
        pytest.skip(f"{codec}: system library not present")


def _payloads():
    rnd = os.urandom(3000)
    text = b"".join(json.dumps({"numericalFeatures": [i * 0.5, i % 7],
                                "categoricalFeatures": [f"c{i % 13}"],
                                "target": 1.0, "operation": "training"}).encode() + b"\n"
                    for i in range(4000))
    return [b"", b"a", rnd, text, rnd + text + rnd]


@pytest.mark.parametrize("codec", CODECS)
def test_codec_roundtrip(codec):
    _need(codec)
    for d in _payloads():
        z = K.compress(codec, d)
        assert K.decompress(codec, z) == d
    text = _payloads()[3]
    assert len(K.compress(codec, text)) < len(text) // 4  # it does compress


def test_snappy_hand_built_streams():
    # raw: len 11 | literal "abcd" | copy (1-byte offset form) len 7 offset 4 (overlapping)
    raw1 = bytes([11, 3 << 2]) + b"abcd" + bytes([(3 << 2) | 1, 4])
    assert K.decompress("snappy", raw1) == b"abcdabcdabc"
    # raw: len 8 | literal "xy" | copy (2-byte offset form) len 6 offset 2
    raw2 = bytes([8, 1 << 2]) + b"xy" + bytes([((6 - 1) << 2) | 2, 2, 0])
    assert K.decompress("snappy", raw2) == b"xyxyxyxy"
    # long literal: tag 60 → one length byte follows (len − 1)
    lit = bytes(range(100))
    raw3 = bytes([100, 60 << 2, 99]) + lit
    assert K.decompress("snappy", raw3) == lit
    # xerial framing (what the Java client writes): magic, version 1, compat 1, blocks
    xer = b"\x82SNAPPY\x00" + struct.pack(">ii", 1, 1)
    for blk in (raw1, raw2):
        xer += struct.pack(">i", len(blk)) + blk
    assert K.decompress("snappy", xer) == b"abcdabcdabc" + b"xyxyxyxy"
    # our encoder writes that framing
    assert K.compress("snappy", b"hello").startswith(b"\x82SNAPPY\x00")
    with pytest.raises(ValueError):
        K.decompress("snappy", bytes([20, 3 << 2]) + b"ab")  # truncated literal


def test_lz4_hand_built_frame():
    _need("lz4")
    xxhash = pytest.importorskip("xxhash")
    data = b"online learning on MI355X " * 20
    flg, bd = 0x60, 0x40  # version 01, independent blocks; max block 64 KiB
    hc = (xxhash.xxh32(bytes([flg, bd]), seed=0).intdigest() >> 8) & 0xFF
    frame = struct.pack("<I", 0x184D2204) + bytes([flg, bd, hc])
    frame += struct.pack("<I", len(data) | 0x80000000) + data  # uncompressed block
    frame += struct.pack("<I", 0)  # end mark
    assert K.decompress("lz4", frame) == data
    with pytest.raises(ValueError):
        K.decompress("lz4", frame[:-6])  # truncated


def test_zstd_hand_built_frame():
    _need("zstd")
    data = b"spoke hub round " * 10  # 160 bytes
    fhd = 0x20  # single segment, 1-byte frame content size, no checksum, no dictionary
    block = (1 | (0 << 1) | (len(data) << 3)).to_bytes(3, "little")  # last, raw, size
    frame = struct.pack("<I", 0xFD2FB528) + bytes([fhd, len(data)]) + block + data
    assert K.decompress("zstd", frame) == data
    with pytest.raises(ValueError):
        K.decompress("zstd", frame[:-10])


def test_gzip_interop_with_python_gzip():
    d = _payloads()[4]
    assert gzip.decompress(K.compress("gzip", d)) == d
    assert K.decompress("gzip", gzip.compress(d)) == d
    assert K.decompress("gzip", gzip.compress(d[:100]) + gzip.compress(d[100:])) == d  # members


def _native_decode(data, offset, max_records=10**6, cap=1 << 24):
    dst = np.empty(cap, dtype=np.uint8)
    n, offs, nxt = K.KafkaBroker._decode_into(data, offset, max_records, dst, cap)
    return [dst[offs[i]:offs[i + 1]].tobytes() for i in range(n)], nxt


@pytest.mark.parametrize("codec", ["none"] + CODECS)
def test_record_batches_python_and_native_agree(codec):
    _need(codec)
    vals = [json.dumps({"i": i, "pad": "x" * (i % 37)}).encode() for i in range(700)]
    data = (K.encode_batch(vals[:300], base_offset=1000, compression=codec)
            + K.encode_batch([b"\0\0\0\0"], base_offset=1299, control=True)
            + K.encode_batch(vals[300:], base_offset=1300, compression=codec))
    py = K.decode_batches(data)
    assert [v for _, v in py] == vals and [o for o, _ in py] == list(range(1000, 1700))
    got, nxt = _native_decode(data, 1000)
    assert got == vals and nxt == 1700
    got, nxt = _native_decode(data, 1250)  # mid-batch start: earlier records skipped
    assert got == vals[250:] and nxt == 1700
    got, nxt = _native_decode(data, 1000, max_records=10)
    assert got == vals[:10] and nxt == 1010
    cap = sum(len(v) for v in vals[:42]) + 5  # the 43rd record does not fit
    got, nxt = _native_decode(data, 1000, cap=cap)
    assert got == vals[:42] and nxt == 1042
    got, nxt = _native_decode(data[:-5], 1000)  # truncated trailing batch ignored
    assert got == vals[:300] and nxt == 1300  # stepped over the control batch too
    bad = bytearray(data)
    bad[60] ^= 0xFF  # inside the first batch's CRC-covered body
    with pytest.raises(IOError, match="CRC"):
        _native_decode(bytes(bad), 1000)


def test_control_batch_alone_advances_the_offset():
    data = K.encode_batch([b"\0\0\0\0"], base_offset=7, control=True)
    assert K.decode_batches(data) == []
    got, nxt = _native_decode(data, 7)
    assert got == [] and nxt == 8


@pytest.mark.parametrize("codec", CODECS)
def test_compressed_topics_through_the_fake_broker(codec):
    _need(codec)
    # a broker without ApiVersions: the client starts at Fetch v4 and must switch to v10
    # when the broker refuses zstd batches to older fetches
    fk = FakeKafka(default_partitions=2, control_every=64, versions="legacy")
    try:
        prod = K.KafkaBroker(f"{fk.addr}?compression={codec}")
        assert prod.codec == K.CODECS[codec]
        prod.create_topic("trainingData", 2)
        recs = [json.dumps({"i": i}).encode() for i in range(600)]
        prod.produce_batch("trainingData", 0, recs[:400])
        prod.produce_batch("trainingData", 1, recs[400:])
        cons = K.KafkaBroker(fk.addr)  # a plain consumer reads any codec
        got, nxt = cons.consume("trainingData", 0, 0, 10**6)
        assert got == recs[:400][:len(got)] and nxt == len(got)
        buf = np.empty(1 << 20, dtype=np.uint8)
        n, offs, nxt = cons.consume_into("trainingData", 1, 0, 1000, buf, len(buf))
        assert n == 200 and nxt == 200
        assert [buf[offs[i]:offs[i + 1]].tobytes() for i in range(n)] == recs[400:]
        # the engine's consumer (partition share of rank 0 of 1) drains both partitions
        c = Consumer(cons, "trainingData", rank=0, world=1)
        seen = []
        for _ in range(20):
            block, offs = c.poll_block(128)
            seen += [block[offs[i]:offs[i + 1]] for i in range(len(offs) - 1)]
        assert sorted(seen) == sorted(recs)
        # zstd needs Fetch v10: the client switches after the broker's error 76
        assert (10 in fk.fetch_versions) == (codec == "zstd")
    finally:
        fk.close()


def test_consume_block_steps_over_a_lone_control_batch():
    _need("zstd")
    class OneShot(K.KafkaBroker):
        def __init__(self, data):
            self.data = data

        def _fetch(self, topic, partition, offset, max_bytes=4 << 20):
            return self.data, offset

    br = OneShot(K.encode_batch([b"\0\0\0\0"], base_offset=3, control=True))
    buf, offs, nxt = br.consume_block("t", 0, 3, 100)
    assert buf == b"" and list(offs) == [0] and nxt == 4
    big = b"y" * 300000  # one record larger than the first guess of the capacity
    br = OneShot(K.encode_batch([big], base_offset=0, compression="zstd"))
    buf, offs, nxt = br.consume_block("t", 0, 0, 100)
    assert buf == big and nxt == 1


@pytest.mark.parametrize("codec", ["none"] + CODECS)
def test_native_batch_encoder_matches_python(codec):
    _need(codec)
    vals = [json.dumps({"mlpId": 1, "prediction": i * 0.25}).encode() for i in range(257)] + [b""]
    block = b"".join(v + b"\n" for v in vals)
    offs = np.zeros(len(vals) + 1, dtype=np.int64)
    np.cumsum([len(v) + 1 for v in vals], out=offs[1:])
    nat = K.encode_lines(np.frombuffer(block, dtype=np.uint8), offs, codec, base_offset=9,
                         ts_ms=777)
    ref = K.encode_batch(vals, base_offset=9, ts_ms=777, compression=codec)
    if codec == "none":
        assert nat == ref  # byte-identical framing, varints and CRC
    assert K.decode_batches(nat) == K.decode_batches(ref)
    assert [v for _, v in K.decode_batches(nat)] == vals


@pytest.mark.parametrize("codec", ["none", "lz4"])
def test_produce_lines_batches_a_tick_block(codec):
    _need(codec)
    fk = FakeKafka(default_partitions=3)
    try:
        br = K.KafkaBroker(fk.addr, compression=codec)
        br.max_batch_bytes = 1000  # force several batches (one Produce each)
        br.create_topic("predictions", 3)
        vals = [json.dumps({"mlpId": 2, "prediction": -1.0, "i": i}).encode() for i in range(500)]
        block = b"".join(v + b"\n" for v in vals)
        offs = np.zeros(len(vals) + 1, dtype=np.int64)
        np.cumsum([len(v) + 1 for v in vals], out=offs[1:])
        br.produce_lines("predictions", block, offs)
        br.produce_lines("predictions", block, offs, partition=2)
        assert fk.logs[("predictions", 0)] == vals
        assert fk.logs[("predictions", 2)] == vals
    finally:
        fk.close()


def test_partitions_fetched_concurrently_on_own_connections():
    _need("zstd")
    import concurrent.futures as cf

    fk = FakeKafka(default_partitions=4)
    try:
        br = K.KafkaBroker(f"{fk.addr}?compression=zstd")
        br.create_topic("trainingData", 4)
        recs = {p: [json.dumps({"p": p, "i": i}).encode() for i in range(300)] for p in range(4)}
        for p in range(4):
            br.produce_batch("trainingData", p, recs[p])
        assert br.parallel_reads
        bufs = [np.empty(1 << 20, dtype=np.uint8) for _ in range(4)]

        def read(p):
            n, offs, nxt = br.consume_into("trainingData", p, 0, 1000, bufs[p], 1 << 20)
            return [bufs[p][offs[i]:offs[i + 1]].tobytes() for i in range(n)], nxt

        with cf.ThreadPoolExecutor(4) as ex:
            out = list(ex.map(read, range(4)))
        for p in range(4):
            assert out[p] == (recs[p], 300)
        assert len(br._conns) >= 2  # one connection per reading thread
        br.close()
    finally:
        fk.close()


@pytest.mark.parametrize("versions,expect", [
    ("classic", {3: 4, 0: 7, 1: 10, 2: 1, 19: 2}),
    ("modern", {3: 4, 0: 7, 1: 10, 2: 1, 19: 2}),   # Kafka 4.0 ranges (KIP-896)
    ("legacy", {3: 1, 0: 3, 1: 4, 2: 1, 19: 0}),    # no ApiVersions: lowest versions
])
def test_api_versions_negotiation(versions, expect):
    fk = FakeKafka(default_partitions=2, versions=versions)
    try:
        br = K.KafkaBroker(fk.addr)
        br.create_topic("requests", 2)
        recs = [json.dumps({"id": i}).encode() for i in range(50)]
        br.produce_batch("requests", 1, recs)
        assert br.end_offset("requests", 1) == 50
        got, nxt = br.consume("requests", 1, 0, 100)
        assert got == recs and nxt == 50
        used = {}
        for api, ver in fk.calls:
            used.setdefault(api, ver)
        for api, ver in expect.items():
            assert used[api] == ver, (api, used)
        br.close()
    finally:
        fk.close()


def test_per_record_consume_steps_over_control_batches():
    """Consumer.poll (requests topic, tools) goes through KafkaBroker.consume: a partition
    that starts with a transaction marker must not stall it."""
    class Log(K.KafkaBroker):
        def __init__(self, data):
            self.data = data

        def _fetch(self, topic, partition, offset, max_bytes=4 << 20):
            return self.data, offset

    vals = [b'{"id": 1}', b'{"id": 2}']
    br = Log(K.encode_batch([b"\0\0\0\0"], base_offset=0, control=True)
             + K.encode_batch(vals, base_offset=1))
    got, nxt = br.consume("requests", 0, 0, 10)
    assert got == vals and nxt == 3
    br = Log(K.encode_batch([b"\0\0\0\0"], base_offset=0, control=True))
    got, nxt = br.consume("requests", 0, 0, 10)
    assert got == [] and nxt == 1


def test_fetch_below_the_retained_log_resumes_at_log_start():
    fk = FakeKafka(default_partitions=1)
    try:
        br = K.KafkaBroker(fk.addr)
        br.create_topic("trainingData", 1)
        recs = [json.dumps({"i": i}).encode() for i in range(30)]
        br.produce_batch("trainingData", 0, recs)
        fk.log_start[("trainingData", 0)] = 10  # retention deleted offsets 0..9
        got, nxt = br.consume("trainingData", 0, 0, 100)
        assert got == recs[10:] and nxt == 30
    finally:
        fk.close()


def test_empty_retained_log_advances_to_log_start():
    """A fetch below a fully-deleted log moves the consumer to the log start for good
    (the next poll must not repeat the failing Fetch + ListOffsets)."""
    class Gone(K.KafkaBroker):
        def __init__(self):
            self.calls = 0

        def _fetch(self, topic, partition, offset, max_bytes=4 << 20):
            self.calls += 1
            return b"", max(offset, 40)  # retention deleted [0, 40): empty log from 40

    br = Gone()
    buf = np.empty(1 << 16, dtype=np.uint8)
    n, offs, nxt = br.consume_into("t", 0, 5, 10, buf, 1 << 16)
    assert n == 0 and nxt == 40
    n, offs, nxt = br.consume_into("t", 0, nxt, 10, buf, 1 << 16)
    assert n == 0 and nxt == 40


def test_consume_into_oversize_record_raises():
    class One(K.KafkaBroker):
        def __init__(self, data):
            self.data = data

        def _fetch(self, topic, partition, offset, max_bytes=4 << 20):
            return self.data, offset

    br = One(K.encode_batch([b"z" * 5000], base_offset=0))
    buf = np.empty(1024, dtype=np.uint8)
    with pytest.raises(IOError, match="does not fit"):
        br.consume_into("t", 0, 0, 10, buf, 1024)
