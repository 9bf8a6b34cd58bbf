"""DIB binary DataInstance records (csrc/host/dib.h, omldm_amd/io/dib.py): a DIB record
parses to exactly what its JSON text parses to (numerical, discrete, categorical slots
in both slot layouts, target, operation, invalid records), mixes with JSON in one block,
and a forecast of it echoes a DataInstance JSON. The GPU parser's decode of the same
records is pinned in tests/test_json_gpu.py."""
import json

import numpy as np
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io import dib
from omldm_amd.io.egress import RawRecords, format_predictions
from omldm_amd.io.parse import parse_block, parse_records
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import join_block

BAD = [
    b'{"numericalFeatures": [1.0], "operation": "training"}',          # no target
    b"EOS",
    b'{"numericalFeatures": [1.0, "x"], "operation": "training", "target": 1}',
    b'{"operation": "forecasting"}',                                     # no features
    b'{"numericalFeatures": null, "categoricalFeatures": [], "operation": "forecasting"}',  # ok
    b'{"discreteFeatures": [3, 4], "operation": "forecasting", "target": null}',           # ok
]


def _spaces():
    return [FeatureSpace(13, 0, 26, 1 << 16), FeatureSpace(3, 2, 4, 1 << 12, field_aware=True)]


def test_dib_parses_like_json_in_both_slot_layouts():
    for space in _spaces():
        recs = [r.encode() for r in synth_json_records(300, space, seed=3)]
        recs += [r.encode() for r in synth_json_records(50, space, seed=4,
                                                        operation="forecasting")]
        recs += BAD
        d = dib.records_to_dib(recs, space.n_numerical, space.n_discrete, space.dc)
        assert all(dib.is_dib(r) and b"\n" not in r for r in d)
        a, opa, va = parse_records(recs, space)
        b, opb, vb = parse_records(d, space)
        assert va == vb == 352 and np.array_equal(opa, opb)
        assert torch.equal(a.num, b.num) and torch.equal(a.cat, b.cat)
        assert torch.equal(torch.nan_to_num(a.y, 7.0), torch.nan_to_num(b.y, 7.0))


def test_dib_block_mixed_with_json_and_newline_framing():
    space = _spaces()[0]
    recs = [r.encode() for r in synth_json_records(200, space, seed=9)]
    d = dib.records_to_dib(recs, space.n_numerical, space.n_discrete, space.dc)
    mixed = [x for pair in zip(recs, d) for x in pair]
    buf = b"".join(r + b"\n" for r in mixed)
    nl = np.flatnonzero(np.frombuffer(buf, dtype=np.uint8) == 10)
    assert len(nl) == len(mixed)  # one newline per record: the payload never holds 0x0A
    offs = np.concatenate([[0], nl + 1]).astype(np.int64)
    bt, op, valid = parse_block(buf, offs, space)
    assert valid == 400
    assert torch.equal(bt.num[0::2], bt.num[1::2]) and torch.equal(bt.cat[0::2], bt.cat[1::2])
    assert torch.equal(bt.y[0::2], bt.y[1::2])


def test_dib_encode_matches_the_converter_and_stuffs_newlines():
    space = FeatureSpace(2, 1, 3, 1 << 10)
    r = dib.encode([10.0 / 256, 2.5], [3], ["a", "b\n", "c"], target=-1.0)
    js = json.dumps({"numericalFeatures": [10.0 / 256, 2.5], "discreteFeatures": [3],
                     "categoricalFeatures": ["a", "b\\n", "c"], "target": -1.0,
                     "operation": "training"})
    assert b"\n" not in r
    a, _, _ = parse_records([js], space)
    b, _, _ = parse_records([dib.records_to_dib([js], 2, 1, 3)[0]], space)
    c, _, _ = parse_records([r], space)
    assert torch.equal(a.num, b.num) and torch.equal(a.num, c.num)
    assert torch.equal(a.cat, b.cat)
    # encode() hashes the decoded string; the JSON parser hashes the raw escaped text
    assert torch.equal(a.cat[:, [0, 2]], c.cat[:, [0, 2]])


def test_dib_forecast_echo_is_datainstance_json():
    space = FeatureSpace(2, 1, 2, 1 << 10)
    r = dib.encode([0.5, -2.0], [7], ["x", "y"], operation="forecasting")
    buf, offs = join_block([r + b"\n", b'{"numericalFeatures": [1.0], "operation": "forecasting"}'])
    raw = RawRecords.from_view(parse_block(buf, offs, space)[0].raw)
    block, _ = format_predictions(raw, 3, np.array([0.25, -1.0], dtype=np.float32))
    out = [json.loads(x) for x in block.decode().splitlines()]
    dp = out[0]["dataPoint"]
    assert dp["numericalFeatures"] == [0.5, -2.0] and dp["discreteFeatures"] == [7.0]
    assert dp["operation"] == "forecasting" and len(dp["categoricalFeatures"]) == 2
    assert all(c.startswith("#") and len(c) == 9 for c in dp["categoricalFeatures"])
    assert out[0]["prediction"] == 0.25 and out[1]["dataPoint"]["numericalFeatures"] == [1.0]
