"""Device holdout routing (csrc/kernels/holdout.hip) == the host reference path."""
import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace, HashedBatch
from omldm_amd.engine.holdout import HoldoutSet

pytestmark = pytest.mark.gpu


def _batch(sp, B, base, dev):
    num = (torch.arange(B * sp.dn, dtype=torch.float32).view(B, sp.dn) + base * 1000)
    cat = (torch.arange(B * sp.dc, dtype=torch.int32).view(B, sp.dc) % 30000).to(sp.cat_dtype)
    y = torch.arange(B, dtype=torch.float32) + base
    return HashedBatch(num.to(dev), cat.to(dev), y.to(dev), cat_span=sp.cat_span)


@pytest.mark.parametrize("field_aware", [False, True])
@pytest.mark.parametrize("size,spokes", [(1, 1), (7, 1), (256, 1), (7, 5), (256, 16)])
def test_device_route_matches_host(cuda, field_aware, size, spokes):
    """The per-spoke device routing (omldm_holdout_route_spokes) moves the same rows
    into the same places as the host index path, ring by ring."""
    sp = FeatureSpace(3, 1, 5, 1 << 16, field_aware=field_aware)
    dev = HoldoutSet(sp, size, cuda, spokes=spokes)
    ref = HoldoutSet(sp, size, "cpu", spokes=spokes)
    rng = np.random.default_rng(size)
    base = 0
    for step in range(40):
        B = int(rng.choice([1, 3, 9, 10, 11, 37, 200, 1500]))
        b = _batch(sp, B, base, "cpu")
        base += B
        out_d = dev.route(b.to(cuda))
        out_h = ref.route(b)
        torch.cuda.synchronize()
        assert torch.equal(out_d.y.cpu(), out_h.y), step
        assert torch.equal(out_d.num.cpu(), out_h.num)
        assert torch.equal(out_d.cat.cpu(), out_h.cat)
        assert out_d.shards == out_h.shards
        for a, b in ((dev.count, ref.count), (dev.head, ref.head), (dev.filled, ref.filled)):
            assert np.array_equal(a, b)
        t_d, t_h = dev.test_set(), ref.test_set()
        assert torch.equal(t_d.y.cpu(), t_h.y)
        assert torch.equal(t_d.cat.cpu(), t_h.cat)
