"""Persistent predict server (gpu-marked): answers match the batch predict kernel for
many points and models, stop/restart works, and the wave exits on its own lifetime."""
import time

import numpy as np
import pytest
import torch

from omldm_amd.api.batch import FeatureSpace
from omldm_amd.io.synthetic import synth_batch
from omldm_amd.ops import linear as L


@pytest.mark.gpu
@pytest.mark.parametrize("field_aware,w_bf16", [(False, False), (True, True)])
def test_persistent_server_matches_predict(cuda, field_aware, w_bf16):
    from omldm_amd.ops.serving import PredictServer

    sp = FeatureSpace(13, 0, 26, 1 << 20, field_aware=field_aware)
    W = torch.randn(3, sp.dim, device=cuda)
    if w_bf16:
        W = W.bfloat16()
    pts = synth_batch(sp, 50, seed=2)
    ref = L.linear_predict(W, pts.to(cuda)).cpu().numpy()
    srv = PredictServer(W, sp.dn, sp.dc, True, sp.cat_span)
    srv.start(lifetime_us=5_000_000)
    for i in range(50):
        got = srv.request(pts.slice(i, i + 1))
        np.testing.assert_allclose(got, ref[i], rtol=1e-4, atol=1e-3)
    srv.stop()
    srv.start(lifetime_us=5_000_000)  # restart after stop
    np.testing.assert_allclose(srv.request(pts.slice(0, 1)), ref[0], rtol=1e-4, atol=1e-3)
    srv.close()


@pytest.mark.gpu
def test_persistent_server_lifetime_exit(cuda):
    from omldm_amd.ops.serving import PredictServer

    sp = FeatureSpace(13, 0, 26, 1 << 16)
    srv = PredictServer(torch.zeros(sp.dim, device=cuda), sp.dn, sp.dc)
    srv.start(lifetime_us=200_000)
    t = time.time()
    while srv.lib.omldm_serve_alive(srv.mb) and time.time() - t < 10:
        time.sleep(0.01)
    assert not srv.lib.omldm_serve_alive(srv.mb)
    srv.stream.synchronize()
    srv.lib.omldm_mailbox_free(srv.mb)
    srv.mb = None
