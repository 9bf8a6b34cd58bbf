"""Tick ingest (engine/ingest.py + csrc/host/logio.cpp): regions of a staging slot read
per partition (in parallel for file logs), one tick ahead on a background thread."""
import json

import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.engine.ingest import TickIngest
from omldm_amd.io.parse import parse_block, parse_records
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import Consumer, FileBroker, MemoryBroker
from omldm_amd.ops import native

SP = FeatureSpace(4, 0, 3, 1 << 12)


def _records(n, seed=0):
    recs = synth_json_records(n, SP, seed=seed)
    out = []
    for i, r in enumerate(recs):
        if i % 7 == 3:  # forecasting points (no target) and some long padding fields
            d = json.loads(r)
            d.pop("target", None)
            d["operation"] = "forecasting"
            d["pad"] = "x" * (i % 50)
            r = json.dumps(d)
        out.append(r)
    return out


def test_index_lines_native():
    buf = np.frombuffer(b'{"a":1}\n{"b":22}\n{"partial"', dtype=np.uint8)
    offs = np.zeros(8, dtype=np.int64)
    n = native.host().omldm_index_lines(buf.ctypes.data, len(buf), 10, offs.ctypes.data)
    assert n == 2 and list(offs[:3]) == [0, 8, 17]
    n = native.host().omldm_index_lines(buf.ctypes.data, len(buf), 1, offs.ctypes.data)
    assert n == 1 and offs[1] == 8


@pytest.mark.parametrize("broker_kind", ["file", "memory"])
@pytest.mark.parametrize("prefetch", [False, True])
def test_tick_ingest_reads_every_record_once(tmp_path, broker_kind, prefetch):
    br = FileBroker(str(tmp_path)) if broker_kind == "file" else MemoryBroker()
    br.create_topic("t", 4)
    br.create_topic("f", 2)
    recs = _records(700)
    for i, r in enumerate(recs):
        br.produce("t" if i % 3 else "f", r, partition=i % 4)
    cons = [Consumer(br, "t"), Consumer(br, "f")]
    ing = TickIngest(cons, batch_size=64, pinned=False, prefetch=prefetch)
    got = []
    for _ in range(200):
        blk = ing.next()
        if blk.n == 0:
            break
        raw = list(blk.raw())
        assert len(raw) == blk.n
        got.extend(r.decode() for r in raw)
        # the parser over the slot (with region gaps) == the parser over clean records
        b1, op1, v1 = parse_block(blk.buf, blk.offs, SP, 2)
        b2, op2, v2 = parse_records(raw, SP, 2)
        assert v1 == v2 and np.array_equal(op1, op2)
        assert torch.equal(b1.cat, b2.cat) and torch.allclose(b1.num, b2.num)
        assert torch.equal(torch.isnan(b1.y), torch.isnan(b2.y))
    ing.close()
    assert sorted(got) == sorted(recs)
    if broker_kind == "file":
        assert all(c.offsets[p] == br.end_offset(c.topic, p) for c in cons for p in c.parts)


def test_empty_prefetch_is_repolled(tmp_path):
    br = FileBroker(str(tmp_path))
    br.create_topic("t", 2)
    c = Consumer(br, "t")
    ing = TickIngest([c], batch_size=16, pinned=False, prefetch=True)
    assert ing.next().n == 0          # starts an (empty) background read
    ing.drain()                       # ... which completes before the records arrive
    for r in _records(10):
        br.produce("t", r)
    assert ing.next().n == 10         # produced between ticks: seen by the next tick
    ing.close()


def test_bulk_produce_block(tmp_path):
    br = FileBroker(str(tmp_path))
    br.create_topic("t", 1)
    br.produce_block("t", 0, b'{"a":1}\n{"a":2}')
    recs, _ = br.consume("t", 0, 0, 10)
    assert recs == [b'{"a":1}', b'{"a":2}']


def test_holdout_closed_forms():
    """The index arithmetic of csrc/kernels/holdout.hip (mirrored here) enumerates the
    non-held / held rows of a batch exactly like the counter rule (pos % 10 >= 8)."""
    from omldm_amd.engine.holdout import HoldoutSet

    def nonheld_row(r, c):
        q = min(c, 8) + r
        return (q // 8) * 10 + q % 8 - c

    def held_row(r, c):
        q = max(c - 8, 0) + r
        return (q // 2) * 10 + 8 + q % 2 - c

    for c in range(10):
        for B in (1, 2, 9, 10, 11, 57, 300):
            pos = (np.arange(B) + c) % 10
            hold = np.flatnonzero(pos >= 8)
            keep = np.flatnonzero(pos < 8)
            assert [nonheld_row(r, c) for r in range(len(keep))] == keep.tolist()
            assert [held_row(r, c) for r in range(len(hold))] == hold.tolist()
            assert HoldoutSet._held_before(c + B) - HoldoutSet._held_before(c) == len(hold)


def test_native_block_fill_matches_python_path(tmp_path, monkeypatch):
    """File-log topics fill a block in one native call (csrc/host/logio.cpp:
    omldm_fill_regions): the same records, slot offsets, true record ends, device-packed
    offsets, segments and consumer positions as the per-region Python path, block after
    block (region gaps included: regions are sized with slack)."""
    br = FileBroker(str(tmp_path))
    br.create_topic("t", 5)
    br.create_topic("f", 2)
    recs = _records(1500, seed=4)
    for i, r in enumerate(recs):
        br.produce("t" if i % 4 else "f", r, partition=i % 5)
    runs = {}
    # one Python reader thread: its regions then update the bytes-per-record estimate in
    # job order, as the native fill does (the slot layout of the next block depends on it)
    monkeypatch.setenv("OMLDM_READERS", "1")
    for native_fill in ("1", "0"):
        monkeypatch.setenv("OMLDM_NATIVE_FILL", native_fill)
        cons = [Consumer(br, "t"), Consumer(br, "f")]
        ing = TickIngest(cons, batch_size=96, pinned=False, prefetch=False)
        assert ing._native_fill == (native_fill == "1")
        ing.stage = True  # the device-packing fields too (filled on the host)
        out = []
        for _ in range(100):
            blk = ing._fill_block(ing._next_slot())
            if blk.n == 0:
                break
            ends = None if blk.ends is None else blk.ends.copy()
            out.append((blk.n, blk.nbytes, blk.offs.copy(), ends,
                        blk.doffs_t.numpy()[: blk.n + 1].copy(), list(blk.segs),
                        blk.dev_nbytes, [r for r in blk.raw()], blk.offsets))
        ing.close()
        runs[native_fill] = out
    a, b = runs["1"], runs["0"]
    assert len(a) == len(b) > 5
    seen = 0
    for x, y in zip(a, b):
        assert x[0] == y[0] and x[1] == y[1] and x[6] == y[6] and x[8] == y[8]
        assert np.array_equal(x[2], y[2]) and np.array_equal(x[4], y[4]) and x[5] == y[5]
        assert (x[3] is None) == (y[3] is None)
        if x[3] is not None:
            assert np.array_equal(x[3], y[3])
        assert x[7] == y[7]
        seen += x[0]
    assert seen == len(recs)


@pytest.mark.parametrize("uniform", [True, False])
def test_split_region_reads_match_one_reader_per_region(tmp_path, monkeypatch, uniform):
    """More readers than regions: each region's first read is cut into ≥ 256 KiB pieces
    read and indexed on their own threads (csrc/host/logio.cpp: omldm_fill_regions) — the
    same blocks as one thread per region, including regions whose hint falls short of
    the records (variable record lengths) and the partial tail at the log's end."""
    br = FileBroker(str(tmp_path))
    br.create_topic("t", 2)
    rng = np.random.default_rng(3)
    for p in range(2):
        lens = np.full(30011, 150) if uniform else rng.integers(20, 400, size=30011)
        br.produce_block("t", p, b"".join(b"x" * int(n - 1) + b"\n" for n in lens))
    runs = {}
    for split in ("1", "0"):
        monkeypatch.setenv("OMLDM_READ_SPLIT", split)  # 1: opt in
        monkeypatch.setenv("OMLDM_READERS", "16")
        cons = [Consumer(br, "t")]
        ing = TickIngest(cons, batch_size=16384, pinned=False, prefetch=False)
        assert ing._native_fill
        ing.stage = True
        out = []
        for _ in range(100):
            blk = ing._fill_block(ing._next_slot())
            if blk.n == 0:
                break
            out.append((blk.n, blk.nbytes, blk.offs.copy(), list(blk.segs), blk.dev_nbytes,
                        blk.doffs_t.numpy()[: blk.n + 1].copy(), [r for r in blk.raw()],
                        blk.offsets))  # (gap bytes between regions are unread: not compared)
        ing.close()
        runs[split] = out
    a, b = runs["1"], runs["0"]
    assert len(a) == len(b) >= 4
    for x, y in zip(a, b):
        assert x[0] == y[0] and x[1] == y[1] and x[3] == y[3] and x[4] == y[4] and x[7] == y[7]
        assert np.array_equal(x[2], y[2]) and np.array_equal(x[5], y[5]) and x[6] == y[6]
    assert sum(x[0] for x in a) == 2 * 30011


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_index_lines_native_matches_python_on_random_blocks(seed):
    """The SIMD record indexer (64 bytes per step, csrc/host/logio.cpp) against a Python
    scan: random record lengths (1..300 bytes, so newlines fall anywhere in a 64-byte
    step), a trailing partial record, record caps that stop mid-step."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 300, size=2000)
    parts = [bytes(rng.integers(0, 9, size=int(n)).astype(np.uint8) + 48) + b"\n" for n in lens]
    blob = b"".join(parts) + b"partial"
    buf = np.frombuffer(blob, dtype=np.uint8)
    ends = [i + 1 for i, c in enumerate(blob) if c == 10]
    for cap in (len(ends) + 5, len(ends), 1337, 1, 64):
        offs = np.zeros(len(ends) + 2, dtype=np.int64)
        n = native.host().omldm_index_lines(buf.ctypes.data, len(buf), cap, offs.ctypes.data)
        want = ends[:cap]
        assert n == len(want) and offs[0] == 0 and list(offs[1:n + 1]) == want
