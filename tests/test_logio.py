"""File-topic reader (csrc/host/logio.cpp): sized first read, incremental top-up reads,
cap and EOF handling — the record index must not depend on how the reads were split."""
import numpy as np
import pytest

from omldm_amd.io.transport import FileBroker


@pytest.mark.parametrize("hint", [0, 1, 100, 5000, 10**9])
def test_read_log_hint_does_not_change_the_records(tmp_path, hint):
    br = FileBroker(str(tmp_path))
    br.create_topic("t", 1)
    rng = np.random.default_rng(0)
    recs = [b'{"x": "' + b"a" * int(rng.integers(1, 300)) + b'"}' for _ in range(2000)]
    with open(tmp_path / "t" / "0.jsonl", "ab") as f:
        f.write(b"".join(r + b"\n" for r in recs) + b'{"partial')  # unterminated tail
    cap = 1 << 20
    dst = np.zeros(cap, dtype=np.uint8)
    off, got = 0, []
    while True:
        n, o, nxt = br.consume_into("t", 0, off, 300, dst, cap, hint=hint)
        if n == 0:
            break
        got += [dst[o[i]:o[i + 1] - 1].tobytes() for i in range(n)]
        assert nxt - off == int(o[n])
        off = nxt
    assert got == recs  # the unterminated tail is left for later
    n, o, nxt = br.consume_into("t", 0, 0, 5, dst, 1000, hint=hint)  # cap limits the records
    assert 0 < n <= 5 and o[n] <= 1000 and nxt == o[n]
