"""GPU JSON parser + feature hashing (csrc/kernels/json_ingest.hip) vs the host C++
scanner: identical features, hashed slots, targets and validity on synthetic and
adversarial records, in both categorical wire formats."""
import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.parse import parse_block
from omldm_amd.io.synthetic import synth_json_records
from omldm_amd.io.transport import join_block

ADVERSARIAL = [
    b'{"numericalFeatures":[1.5,-2,3e2],"categoricalFeatures":["a","b"],"target":1,'
    b'"operation":"training"}',
    b'{"numericalFeatures":[1e400,-1e-400,0],"target":-1,"operation":"training"}',
    b'{"numericalFeatures":[1,2,',
    b'',
    b'   ',
    b'EOS',
    b'{"operation":"forecasting","categoricalFeatures":["x","y","z\\"q","w","v"]}',
    b'{"numericalFeatures":[1,2,3,4,5,6,7,8,9,10,11,12,13,14,15],"target":0.5,'
    b'"operation":"training"}',
    b'{"discreteFeatures":[1,2],"target":"oops","operation":"training"}',
    b'{"numericalFeatures":[],"categoricalFeatures":[],"target":null,"operation":"training"}',
    b'{"id":{"nested":[1,{"a":"]"}]},"numericalFeatures":[0.25],"target":2,'
    b'"operation":"training","extra":[true,false,null]}',
    b'{"numericalFeatures":null,"discreteFeatures":[3,4],"categoricalFeatures":null,'
    b'"target":1.25e-3,"operation":"training"}',
    b'{"numericalFeatures":[123456789012345678901234,3.14159265358979323846],"target":1,'
    b'"operation":"training"}',
    b'{}',
    b'{"numericalFeatures":[1],"operation":"unknown"}',
]


@pytest.mark.gpu
@pytest.mark.parametrize("field_aware", [False, True])
def test_gpu_parser_matches_host(cuda, field_aware):
    from omldm_amd.ops.ingest import GpuJsonParser

    sp = FeatureSpace(13, 2, 26, 1 << 20, field_aware=field_aware)
    recs = [r.encode() for r in synth_json_records(3000, sp, seed=9)]
    recs += ADVERSARIAL * 3
    # a record with a huge skipped field: its 64-record group exceeds the wave's LDS stage
    # and is parsed from global memory (the other groups from LDS)
    recs.insert(1000, b'{"numericalFeatures":[7],"blob":"' + b"z" * 50000 + b'","target":1,'
                b'"operation":"training"}')
    buf, offs = join_block(recs)
    hb, hop, hval = parse_block(buf, offs, sp, 4)
    gb, gop, gval = GpuJsonParser(cuda).parse(buf, offs, sp)
    torch.cuda.synchronize()
    assert np.array_equal(gop.cpu().numpy(), hop)
    c = gval.cpu().tolist()
    assert c[0] + c[1] == hval and c[2] == len(recs) - hval
    assert c[0] == int((hop == 0).sum()) and c[1] == int((hop == 1).sum())
    ok = torch.from_numpy(hop >= 0)
    assert torch.equal(gb.num.cpu()[ok], hb.num[ok])
    assert torch.equal(gb.cat.cpu()[ok], hb.cat[ok])
    assert torch.equal(torch.nan_to_num(gb.y.cpu()[ok], nan=-7.0),
                       torch.nan_to_num(hb.y[ok], nan=-7.0))


@pytest.mark.gpu
def test_gpu_parser_exact_size_buffer_and_group_edges(cuda):
    """The staged kernel never reads past the last record (an exact-size device buffer),
    and record counts that are not multiples of the 64-record group parse identically."""
    from omldm_amd.ops.ingest import json_parse

    sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=True)
    for n in (1, 63, 65, 200):
        recs = [r.encode() for r in synth_json_records(n, sp, seed=n)]
        buf, offs = join_block(recs)
        hb, hop, _ = parse_block(buf, offs, sp, 2)
        d = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(cuda)  # exact size
        o = torch.from_numpy(offs).to(cuda)
        num = torch.empty((n, sp.dn), dtype=torch.float32, device=cuda)
        cat = torch.empty((n, sp.dc), dtype=sp.cat_dtype, device=cuda)
        y = torch.empty(n, dtype=torch.float32, device=cuda)
        op = torch.empty(n, dtype=torch.int8, device=cuda)
        cnt = torch.zeros(3, dtype=torch.int32, device=cuda)
        json_parse(d, o, n, sp, num, cat, y, op, cnt, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(op.cpu().numpy(), hop)
        ok = torch.from_numpy(hop >= 0)
        assert torch.equal(num.cpu()[ok], hb.num[ok]) and torch.equal(cat.cpu()[ok], hb.cat[ok])


@pytest.mark.gpu
@pytest.mark.parametrize("field_aware", [False, True])
def test_gpu_parser_decodes_dib_like_the_json(cuda, field_aware):
    """DIB records (omldm_amd/io/dib.py) interleaved with JSON in one block: the GPU
    parser's rows equal the host parser's rows of the JSON originals."""
    from omldm_amd.io import dib
    from omldm_amd.ops.ingest import GpuJsonParser

    sp = FeatureSpace(13, 2, 26, 1 << 20, field_aware=field_aware)
    recs = [r.encode() for r in synth_json_records(2000, sp, seed=5)] + ADVERSARIAL * 2
    d = dib.records_to_dib(recs, sp.n_numerical, sp.n_discrete, sp.dc)
    mixed = [x for i, pair in enumerate(zip(recs, d)) for x in (pair if i % 3 else pair[::-1])]
    buf, offs = join_block([r + b"\n" for r in mixed])
    hb, hop, hval = parse_block(*join_block(recs), sp, 4)
    gb, gop, gval = GpuJsonParser(cuda).parse(buf, offs, sp)
    torch.cuda.synchronize()
    g = gop.cpu().numpy()
    assert np.array_equal(g[0::2], hop) and np.array_equal(g[1::2], hop)
    assert gval.cpu().tolist()[:2] == [2 * int((hop == 0).sum()), 2 * int((hop == 1).sum())]
    ok = torch.from_numpy(hop >= 0)
    for k in (0, 1):
        assert torch.equal(gb.num.cpu()[k::2][ok], hb.num[ok])
        assert torch.equal(gb.cat.cpu()[k::2][ok], hb.cat[ok])
        assert torch.equal(torch.nan_to_num(gb.y.cpu()[k::2][ok], nan=-7.0),
                           torch.nan_to_num(hb.y[ok], nan=-7.0))


@pytest.mark.gpu
def test_gpu_pull_copy_segments_one_launch():
    """Several pinned-host → HBM segments in one launch (csrc/kernels/ingest.hip:
    pull_copy_segs_kernel): odd lengths (bytewise tails), the engine's slot layout."""
    from omldm_amd.ops.ingest import pull_copy_segs

    dev = torch.device("cuda", 0)
    host = torch.randint(0, 256, (1 << 20,), dtype=torch.uint8).pin_memory()
    out = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    segs = [(0, 0, 1000), (4096, 1008, 77777), (200000, 90000, 16), (300000, 100000, 5),
            (400016, 200000, 333331)]
    pull_copy_segs([(host.data_ptr() + h, out.data_ptr() + d, n) for h, d, n in segs], 64)
    torch.cuda.synchronize()
    o = out.cpu()
    for h, d, n in segs:
        assert torch.equal(o[d:d + n], host[h:h + n])
    untouched = torch.ones(1 << 20, dtype=torch.bool)
    for h, d, n in segs:
        untouched[d:d + n] = False
    assert int(o[untouched].abs().sum()) == 0
