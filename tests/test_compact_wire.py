"""Compact wire format (field-aware uint16 categorical slots): CPU ↔ dense ↔ HIP."""
import json

import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.parse import hash_categorical, parse_records
from omldm_amd.io.synthetic import synth_batch
from omldm_amd.ops import linear as L

SP = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)


def test_span_and_dtype():
    assert SP.cat_span == 32767 and SP.cat_dtype == torch.int16
    b = synth_batch(SP, 100, seed=4)
    assert b.cat.dtype == torch.int16 and b.cat_span == SP.cat_span
    slot, sign, valid = b.cat_slots()
    assert valid.all()
    f = torch.arange(26).unsqueeze(0)
    assert ((slot >= SP.dn + f * SP.cat_span) & (slot < SP.dn + (f + 1) * SP.cat_span)).all()
    assert set(sign.unique().tolist()) <= {-1.0, 1.0}


def test_predict_matches_dense_compact():
    b = synth_batch(SP, 64, seed=6)
    W = torch.randn(2, SP.dim)
    out = L.linear_predict(W, b)
    X = b.dense(SP.dim)
    X[:, SP.dim - 1] = 1.0
    np.testing.assert_allclose(out.numpy(), (X @ W.T).numpy(), rtol=1e-4, atol=1e-4)


def test_parse_compact_matches_hash():
    rec = {"numericalFeatures": [0.5] * 13, "categoricalFeatures": [f"t{j}" for j in range(26)],
           "target": 1.0, "operation": "training"}
    b, op, n = parse_records([json.dumps(rec)], SP)
    assert n == 1 and op[0] == 0
    expect = [hash_categorical(f"t{j}", j, SP) for j in range(26)]
    got = (b.cat[0].long() & 0xFFFF).tolist()
    assert got == [e & 0xFFFF for e in expect]


def test_round_learns_compact():
    w = torch.zeros(SP.dim)
    d = torch.zeros(SP.dim + 2)
    for r in range(4):
        L.linear_round(w, synth_batch(SP, 8192, start=r * 8192), 512, 16, d, None,
                       L.LinearRule(), 1.0)
        L.linear_apply(w, None, d)
    t = synth_batch(SP, 4000, start=10**8)
    acc = float(((L.linear_predict(w, t) >= 0).float() * 2 - 1 == t.y).float().mean())
    assert acc > 0.7


@pytest.mark.gpu
def test_hip_round_compact_matches_cpu(cuda):
    S, R = 64, 32
    b = synth_batch(SP, S * R, seed=12)
    b.num = b.num.bfloat16().float()  # same inputs as the bf16 wire below
    w = torch.randn(SP.dim) * 0.01
    d_cpu = torch.zeros(SP.dim + 2)
    L.linear_round(w, b, R, S, d_cpu, None, L.LinearRule(), 1.0)
    bg = b.to(cuda)
    bg.num = bg.num.bfloat16().contiguous()
    d_gpu = torch.zeros(SP.dim + 2, device=cuda)
    st = torch.zeros(S, 6, device=cuda)
    L.linear_round(w.to(cuda), bg, R, S, d_gpu, st, L.LinearRule(), 1.0, log2cap=11)
    assert float(st[:, 5].sum()) == 0.0
    np.testing.assert_allclose(d_gpu.cpu().numpy(), d_cpu.numpy(), rtol=2e-3, atol=2e-4)
    out = L.linear_predict(w.to(cuda), bg)
    ref = L.linear_predict(w, b)
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
