"""One engine over several replicas (tm_open_devices, VERDICT r1 "multi-GPU
engine in the C-ABI").  The box has one GPU, so the replicas share device 0:
host batches are still cut into one slice per replica and run by one worker
per replica, exactly as across 8 GPUs.  Results must equal O1 and the
single-replica engine, for match/1, match_routes/1 and aggre/1, through the
batch API and the micro-batcher's lanes."""
import os
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402

pytestmark = pytest.mark.gpu


def _o1(fb, fo):
    from oracle import O1
    o = O1()
    o.insert_many(fb, fo)
    return o


@pytest.mark.parametrize("replicas", [2, 3, 4])
def test_replicas_match_equals_o1(gpu_device, replicas):
    fb, fo = W.filters(2, n=200_000)
    tb, to = W.topics(2, n=50_000)
    e = Engine(devices=[gpu_device] * replicas, filters_hint=200_000)
    assert e.replicas == replicas
    e.insert_many(fb, fo)
    o1 = _o1(fb, fo)
    oc, oo, oi = o1.match_ids(tb, to, threads=8)
    e.set_stats(True)
    counts, offs, ids = e.match_batch(tb, to)
    st = e.last_stats()
    e.set_stats(False)
    assert np.array_equal(counts, oc) and np.array_equal(offs, oo) and np.array_equal(ids, oi)
    assert st["topics"] == 50_000 and st["matches"] == int(oo[-1])
    # fewer topics than replicas, and a caller-sized output that overflows
    for k in (1, 2, replicas + 1):
        c, o, i = e.match_batch(tb[: int(to[k])], to[: k + 1])
        assert np.array_equal(i, oi[: int(oo[k])])
    from emqx_amd import _lib as L
    with pytest.raises(L.TopicMatchError) as ex:
        e.match_batch(tb, to, out_cap=int(oo[-1]) - 1)
    assert ex.value.code == L.TM_ENOSPC
    e.close()


def test_replicas_routes_and_deliveries_equal_single(gpu_device):
    from emqx_amd.emqx_router import Router
    fb, fo = W.filters(1)
    tb, to = W.topics(1, n=30_000)
    topics = W.unpack(tb, to)
    dests = ["n1", "n2", ("g1", "n1"), ("g1", "n2"), ("g2", "n3")]
    rng = np.random.default_rng(4)
    engines = [Engine(device=gpu_device), Engine(devices=[gpu_device] * 3)]
    routers = [Router(x, node="n1") for x in engines]
    for i, f in enumerate(W.unpack(fb, fo)):
        for d in rng.choice(len(dests), size=int(rng.integers(1, 3)), replace=False):
            for r in routers:
                r.add_route(f, dests[d])
    for t in topics[::11]:
        for r in routers:
            r.add_route(t, "n3")
    a = engines[0].match_routes_batch(tb, to)
    b = engines[1].match_routes_batch(tb, to)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert routers[0].match_deliveries_many(topics, tagged=True) == routers[1].match_deliveries_many(topics, tagged=True)
    for x in engines:
        x.close()


def test_batcher_lanes_over_replicas(gpu_device):
    from emqx_amd.batcher import Batcher
    fb, fo = W.filters(2, n=100_000)
    tb, to = W.topics(2, n=40_000)
    topics = W.unpack(tb, to)
    e = Engine(devices=[gpu_device] * 2)
    e.insert_many(fb, fo)
    oc, oo, oi = _o1(fb, fo).match_ids(tb, to, threads=8)
    b = Batcher(e, max_topics=2500, deadline_us=300, lanes_per_replica=3)
    got = [None] * len(topics)

    def producer(k):
        for t in range(k, len(topics), 6):
            def cb(status, ids, dests, t=t):
                assert status == 0
                got[t] = ids
            b.submit(topics[t], cb)
    ts = [threading.Thread(target=producer, args=(k,)) for k in range(6)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    b.flush()
    st = b.stats()
    b.close()
    assert st["topics"] == len(topics) and st["failed_batches"] == 0 and st["batches"] >= 10
    for t in range(len(topics)):
        assert got[t] == [int(x) for x in oi[oo[t]:oo[t + 1]]], t
    e.close()


def test_device_api_on_replicated_engine(gpu_device):
    import torch
    fb, fo = W.filters(1)
    tb, to = W.topics(1, n=5000)
    e = Engine(devices=[gpu_device, gpu_device])
    e.insert_many(fb, fo)
    oc, oo, oi = _o1(fb, fo).match_ids(tb, to, threads=4)
    dev = torch.device("cuda", gpu_device)
    n = len(to) - 1
    d_b = torch.from_numpy(tb.copy()).to(dev)
    d_o = torch.from_numpy(to.view(np.int64).copy()).to(dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)
    o = torch.empty(n + 1, dtype=torch.int64, device=dev)
    t = torch.zeros(1, dtype=torch.int64, device=dev)
    i = torch.empty(int(oo[-1]) + 8, dtype=torch.int32, device=dev)
    e.match_batch_device(d_b, d_o, n, int(to[-1]), c, o, i, i.numel(), t)
    torch.cuda.synchronize()
    assert int(t.item()) == int(oo[-1])
    assert np.array_equal(i[: int(oo[-1])].cpu().numpy().view(np.uint32), oi)
    e.close()
