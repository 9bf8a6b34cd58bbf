"""Native prediction egress (csrc/host/egress.cpp) == Prediction.to_json semantics."""
import json
import math

import numpy as np

from omldm_amd.api.schemas import Prediction
from omldm_amd.io.egress import RawRecords, format_predictions
from omldm_amd.io.parse import RawView
from omldm_amd.io.transport import FileBroker, MemoryBroker, join_block


def _same(a, b):
    if isinstance(a, float) and math.isnan(a):
        return isinstance(b, float) and math.isnan(b)
    return a == b


def test_format_matches_python_prediction():
    recs = [json.dumps({"numericalFeatures": [i * 0.5, -1e-7], "categoricalFeatures": ["a", "é"],
                        "operation": "forecasting"}).encode() for i in range(9)]
    recs[3] = b"  " + recs[3] + b" \n"
    buf, offs = join_block(recs)
    preds = np.array([1.0, -1.0, 0.1, 123456789.0, 1e-30, float("nan"), float("inf"),
                      -float("inf"), 3.5e20], dtype=np.float32)
    block, loffs = format_predictions(RawRecords.from_view(RawView(buf, offs)), 7, preds)
    lines = block.split(b"\n")[:-1]
    assert len(lines) == 9 and loffs[-1] == len(block)
    for i, line in enumerate(lines):
        got = json.loads(line)
        want = json.loads(Prediction(7, recs[i], float(preds[i])).to_json())
        assert got["mlpId"] == want["mlpId"] and got["dataPoint"] == want["dataPoint"]
        assert _same(got["prediction"], want["prediction"]), (got, want)
        # the number is printed like json.dumps prints the same Python float
        assert line.endswith((json.dumps(float(preds[i])) + "}").encode())


def test_subset_and_gapped_ends():
    recs = [b'{"x": 1}', b'{"x": 2}', b'{"x": 3}']
    buf = b'{"x": 1}\nGARBAGE{"x": 2}\n{"x": 3}\n'
    offs = np.array([0, 16, 25, 34])
    ends = np.array([9, 25, 34])  # record 0 is followed by a region gap
    raw = RawRecords.from_view(RawView(buf, offs, ends), np.array([0, 2]))
    block, _ = format_predictions(raw, 1, np.array([1.0, 0.0], dtype=np.float32))
    got = [json.loads(x) for x in block.split(b"\n")[:-1]]
    assert [g["dataPoint"]["x"] for g in got] == [1, 3]


def test_produce_lines_file_and_memory(tmp_path):
    block, offs = format_predictions(RawRecords.from_view([b'{"a": 1}', b'{"a": 2}']), 3,
                                     np.array([0.5, 2.0], dtype=np.float32))
    for br in (FileBroker(str(tmp_path)), MemoryBroker()):
        br.create_topic("p", 1)
        br.produce_lines("p", block, offs)
        recs, _ = br.consume("p", 0, 0, 10)
        assert [json.loads(r)["prediction"] for r in recs] == [0.5, 2.0]


def test_chunked_formatting_and_writer_order(tmp_path):
    from omldm_amd.io.egress import EgressWriter, format_predictions_chunks

    recs = [json.dumps({"i": i}).encode() for i in range(1000)]
    raw = RawRecords.from_view(recs)
    preds = np.arange(1000, dtype=np.float32)
    chunks = format_predictions_chunks(raw, 2, preds, chunk=97)
    assert len(chunks) == 11
    br = FileBroker(str(tmp_path))
    br.create_topic("p", 1)
    w = EgressWriter(br)
    for block, offs in chunks:
        w.submit("p", block, offs)
    w.close()
    got, _ = br.consume("p", 0, 0, 5000)
    assert [json.loads(r)["dataPoint"]["i"] for r in got] == list(range(1000))
    assert [json.loads(r)["prediction"] for r in got] == [float(i) for i in range(1000)]
