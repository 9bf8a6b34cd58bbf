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
@pytest.mark.parametrize("size", [1, 7, 256])
def test_device_route_matches_host(cuda, field_aware, size):
    sp = FeatureSpace(3, 1, 5, 1 << 16, field_aware=field_aware)
    dev = HoldoutSet(sp, size, cuda)
    ref = HoldoutSet(sp, size, "cpu")
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
        assert (dev.count, dev.head, dev.filled) == (ref.count, ref.head, ref.filled)
        t_d, t_h = dev.test_set(), ref.test_set()
        assert torch.equal(t_d.y.cpu(), t_h.y)
        assert torch.equal(t_d.cat.cpu(), t_h.cat)
