"""Fused hub-merge kernels (csrc/kernels/merge.hip) vs the PyTorch fp32 reference."""
import pytest
import torch

from omldm_amd.ops import merge as M


def _vecs(n, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(n, generator=g) for _ in range(k)]


def test_cpu_merge_ops_semantics():
    x, E, sh = _vecs(1001, 3)
    out = M.drift_norms(x, E, 2.0)
    torch.testing.assert_close(out[0], ((x - E) * 2).pow(2).sum())
    sent, buf, sh0 = torch.empty_like(x), torch.empty_like(x), sh.clone()
    M.async_push(x, E, sh, sent, buf)
    torch.testing.assert_close(sent, x - E - sh0)
    torch.testing.assert_close(sh, sh0 + sent)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 7, 4096, 1_000_003])
def test_hip_merge_ops(cuda, n):
    x, E, d, sh, c = _vecs(n, 5, seed=n)
    g = lambda t: t.clone().to(cuda)  # noqa: E731
    # drift norms
    out = M.drift_norms(g(x), g(E), 3.0).cpu()
    ref = M.drift_norms(x, E, 3.0)
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3)
    # fold + reload
    Eg, xg = g(E), g(x)
    M.fold_reload(Eg, g(d), 0.25, xg)
    Ec, xc = E.clone(), x.clone()
    M.fold_reload(Ec, d, 0.25, xc)
    torch.testing.assert_close(Eg.cpu(), Ec)
    torch.testing.assert_close(xg.cpu(), xc)
    # elastic pre/post
    xg, cg, dg, sg = g(x), g(c), torch.empty(n, device=cuda), torch.empty(n, device=cuda)
    M.elastic_pre(xg, cg, dg, sg)
    sg.mul_(2.0)
    M.elastic_post(xg, cg, dg, sg, 0.1)
    xc, cc, dc, sc = x.clone(), c.clone(), torch.empty(n), torch.empty(n)
    M.elastic_pre(xc, cc, dc, sc)
    sc.mul_(2.0)
    M.elastic_post(xc, cc, dc, sc, 0.1)
    torch.testing.assert_close(xg.cpu(), xc)
    torch.testing.assert_close(cg.cpu(), cc)
    # async push / pull
    xg, Eg, shg = g(x), g(E), g(sh)
    sent, buf = torch.empty(n, device=cuda), torch.empty(n, device=cuda)
    M.async_push(xg, Eg, shg, sent, buf)
    buf.mul_(3.0)
    M.async_pull(xg, Eg, shg, sent, buf, 0.5)
    xc, Ec, shc = x.clone(), E.clone(), sh.clone()
    s2, b2 = torch.empty(n), torch.empty(n)
    M.async_push(xc, Ec, shc, s2, b2)
    b2.mul_(3.0)
    M.async_pull(xc, Ec, shc, s2, b2, 0.5)
    for a, b in ((xg, xc), (Eg, Ec), (shg, shc)):
        torch.testing.assert_close(a.cpu(), b, rtol=1e-5, atol=1e-5)
