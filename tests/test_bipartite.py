"""Bipartite topology: messages + byte accounting, buffers, wrappers, and the golden
message-passing protocols under seeded delivery interleavings."""
import numpy as np
import pytest

from omldm_amd.engine.bipartite import (BufferingWrapper, GenericWrapper, SynchronousWorker,
                                        build_topology, run_stream)
from omldm_amd.engine.network import (RPC, HubMessage, LocalNetwork, NetworkDescriptor, NodeId,
                                      NodeType, SpokeMessage, payload_size)
from omldm_amd.utils.dataset import DataSet, IntWrapper, integer_parsing


def test_dataset_fifo():
    d = DataSet(3)
    assert [d.append(i) for i in range(5)] == [None, None, None, 0, 1]
    assert d.data_buffer == [2, 3, 4] and d.length == 3
    assert d.pop() == 2 and d.length == 2
    e = DataSet(2, [7, 8])
    d.merge([e])
    assert d.data_buffer == [3, 4, 7, 8] and d.get_max_size() == 4
    d.clear()
    assert d.is_empty() and not d.non_empty()
    assert DataSet.from_state(DataSet(5, [1, 2]).state_dict()).data_buffer == [1, 2]


def test_small_utils():
    w = IntWrapper(3)
    w.set_int(w.get_int() + 1)
    assert w.get_int() == 4
    assert integer_parsing({"HubParallelism": "4"}, "HubParallelism", 1) == 4
    assert integer_parsing({"HubParallelism": "x"}, "HubParallelism", 1) == 1
    assert integer_parsing(None, "k", 7) == 7


def test_message_sizes_and_fanout():
    s, h = NodeId(NodeType.SPOKE, 1), NodeId(NodeType.HUB, 0)
    v = np.zeros(10, np.float32)
    m = SpokeMessage(3, RPC.PUSH, s, h, v)
    assert m.get_size() == 4 + 4 + 8 + 8 + 40
    assert SpokeMessage(-1, None, s, None).is_heartbeat
    dests = [NodeId(NodeType.SPOKE, i) for i in range(4)]
    hm = HubMessage(3, [RPC.UPDATE] * 4, h, dests, v)
    assert hm.get_size() == 4 + 16 + 8 + 32 + 40
    assert hm.legacy_size() == 4 * hm.get_size()
    assert [c.destination for c in hm.fan_out(4)] == dests
    term = HubMessage()
    assert term.is_termination and len(term.fan_out(5)) == 5
    assert payload_size([v, b"ab", 1.0]) == 40 + 2 + 8


def test_generic_wrapper_drains_cache_on_create():
    net = LocalNetwork(NetworkDescriptor(0, 1, 1))
    got = []

    class H:
        def receive_msg(self, src, rpc, data):
            got.append(data)

    gw = GenericWrapper(NodeId(NodeType.HUB, 0), net)
    gw.receive_msg(None, RPC.PUSH, 1)
    gw.receive_msg(None, RPC.PUSH, 2)
    assert got == []
    gw.create(H())
    assert got == [1, 2]
    gw.receive_msg(None, RPC.PUSH, 3)
    assert got == [1, 2, 3]


def test_buffering_wrapper_replays_in_order():
    net = LocalNetwork(NetworkDescriptor(0, 1, 1))
    seen = []

    def fit(w, p):
        seen.append(p)
        return w

    nid = NodeId(NodeType.SPOKE, 0)
    wk = SynchronousWorker(nid, net, np.zeros(2), fit, batch=2)
    bw = BufferingWrapper(nid, net, wk)
    for p in range(5):
        bw.receive_tuple(p)
    assert seen == [0, 1] and bw.buffer.data_buffer == [2, 3, 4]
    bw.receive_msg(NodeId(NodeType.HUB, 0), RPC.UPDATE, np.ones(2))
    # unblocked → replays 2,3 then blocks again at the next round end
    assert seen == [0, 1, 2, 3] and bw.buffer.data_buffer == [4]


def _pa_fit(w, p):
    x, y = p
    loss = max(0.0, 1 - y * float(w @ x))
    return w + min(1.0, loss / float(x @ x)) * y * x if loss > 0 else w


def _stream(n, d=6, seed=0):
    rng = np.random.default_rng(seed)
    wt = rng.standard_normal(d)
    out = []
    for _ in range(n):
        x = rng.standard_normal(d)
        out.append((x, 1.0 if x @ wt >= 0 else -1.0))
    return out, wt


def test_sync_golden_is_model_averaging():
    P, B = 3, 4
    pts, _ = _stream(P * B * 2, seed=1)
    net, hub, spokes = build_topology("Synchronous", P, np.zeros(6), _pa_fit, batch=B, seed=5)
    run_stream(net, spokes, pts, shard=lambda i: (i // B) % P, deliver_every=10**9)
    # reference computation: round r, worker k trains on its B points from the average
    w = np.zeros(6)
    for r in range(2):
        locs = []
        for k in range(P):
            wk = w.copy()
            for j in range(B):
                wk = _pa_fit(wk, pts[r * P * B + k * B + j])
            locs.append(wk)
        w = np.mean(locs, axis=0)
    np.testing.assert_allclose(hub.node.w, w, rtol=1e-12)
    for s in spokes:
        np.testing.assert_allclose(s.worker.w, w, rtol=1e-12)
    # 2 rounds × (P pushes + 1 broadcast)
    assert net.messages == 2 * (P + 1)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_ssp_staleness_bound_under_interleavings(seed):
    P, s = 4, 2
    pts, wt = _stream(2000, seed=seed)
    net, hub, spokes = build_topology("SSP", P, np.zeros(6), _pa_fit, batch=5, seed=seed,
                                      staleness=s)
    rng = np.random.default_rng(seed)
    skew = rng.permutation(P)  # uneven shard rates: worker skew[0] gets most data
    weights = np.array([8, 4, 2, 1])[skew]
    shard = rng.choice(P, size=len(pts), p=weights / weights.sum())
    run_stream(net, spokes, pts, shard=lambda i: int(shard[i]), deliver_every=3)
    assert hub.node.max_gap <= s
    acc = np.mean([np.sign(x @ hub.node.w) == y for x, y in pts[-500:]])
    assert acc > 0.85


def test_async_converges_and_easgd_contracts():
    P = 4
    pts, _ = _stream(3000, seed=7)
    net, hub, spokes = build_topology("Asynchronous", P, np.zeros(6), _pa_fit, batch=5, seed=3)
    run_stream(net, spokes, pts, shard=lambda i: i % P, deliver_every=2)
    acc = np.mean([np.sign(x @ hub.node.w) == y for x, y in pts[-500:]])
    assert acc > 0.85
    net, hub, spokes = build_topology("EASGD", P, np.zeros(6), _pa_fit, batch=5, seed=3,
                                      alpha=0.2)
    run_stream(net, spokes, pts, shard=lambda i: i % P, deliver_every=2)
    spread = max(np.linalg.norm(s.worker.w - hub.node.w) for s in spokes)
    scale = np.linalg.norm(hub.node.w)
    assert scale > 0 and spread < scale
