"""Micro-batcher on the GPU: 4 publisher threads submit single topics; every
callback's list must equal the batch API's result for that topic (ordered
emqx_trie:match/1 ids, or match_routes/1 routes), whatever batch it rode in."""
import os
import sys
import threading

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402
from emqx_amd.batcher import Batcher  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("routes,cbt", [(False, 0), (True, 0), ("deliveries", 0), (False, 3), ("deliveries", 2)])
def test_batcher_results_equal_batch_api(gpu_device, routes, cbt):
    """cbt > 0: callback threads share each batch's callbacks with its lane
    (batches of up to 20K topics: parts of >= 8192)"""
    fb, fo = W.filters(1)
    tb, to = W.topics(1, n=40000)
    topics = W.unpack(tb, to)
    e = Engine(device=gpu_device)
    if routes:
        for i, f in enumerate(W.unpack(fb, fo)):
            e.route_add(f, b"node%d" % (i % 3))
        for t in topics[::5]:
            e.route_add(t, b"direct")
        if routes == "deliveries":
            for i, f in enumerate(W.unpack(fb, fo)[::3]):     # $share members: {Group, Node}
                e.dest_target(b"grp%d|node%d" % (i % 4, i % 3), Engine.TARGET_GROUP, b"grp%d" % (i % 4))
                e.route_add(f, b"grp%d|node%d" % (i % 4, i % 3))
            counts, offs, src, dst = e.match_deliveries_batch(tb, to)
            want = [(list(src[offs[t]:offs[t] + counts[t]]), list(dst[offs[t]:offs[t] + counts[t]]))
                    for t in range(len(topics))]
        else:
            counts, offs, src, dst = e.match_routes_batch(tb, to)
            want = [(list(src[offs[t]:offs[t + 1]]), list(dst[offs[t]:offs[t + 1]])) for t in range(len(topics))]
    else:
        e.insert_many(fb, fo)
        counts, offs, ids = e.match_batch(tb, to)
        want = [(list(ids[offs[t]:offs[t + 1]]), None) for t in range(len(topics))]
        # the batch API itself against O1 (no self-comparison only)
        from oracle import O1
        o1 = O1()
        o1.insert_many(fb, fo)
        oc, oo, oi = o1.match_ids(tb, to, threads=8)
        filters = W.unpack(fb, fo)
        for t in range(0, len(topics), 7):
            assert [e.filter_bytes(int(x)) for x in want[t][0]] == [filters[j] for j in oi[oo[t]:oo[t + 1]]], t
    b = Batcher(e, max_topics=20000 if cbt else 3000, deadline_us=500, routes=routes is True,
                deliveries=routes == "deliveries", callback_threads=cbt)
    got = [None] * len(topics)

    def producer(k):
        for t in range(k, len(topics), 4):
            def cb(status, ids, dests, t=t):
                assert status == 0
                got[t] = (ids, dests)
            b.submit(topics[t], cb)
    ts = [threading.Thread(target=producer, args=(k,)) for k in range(4)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    b.flush()
    st = b.stats()
    b.close()
    assert st["topics"] == len(topics) and st["failed_batches"] == 0 and st["batches"] >= (2 if cbt else 5)
    for t in range(len(topics)):
        ids, dests = got[t]
        assert [int(x) for x in want[t][0]] == ids, t
        if routes:
            assert [int(x) for x in want[t][1]] == dests, t
    assert sum(len(g[0]) for g in got) > 100_000
    e.close()


def test_routes_and_deliveries_batchers_concurrently(gpu_device):
    """a routes batcher and a deliveries batcher on ONE engine
    (the NIF opens both), fed at once from 4 threads each; both result sets
    must equal the batch API, which is pinned to the oracle (a sample is
    checked against oracle/pytrie.py directly as well)"""
    import random
    from emqx_amd.emqx_router import Router
    from oracle import pytrie
    fb, fo = W.filters(1, n=4000)
    tb, to = W.topics(1, n=20000)
    topics = W.unpack(tb, to)
    e = Engine(device=gpu_device)
    r, o = Router(e, node="n1"), pytrie.RouteTable()
    rng = random.Random(3)
    dests = ["n1", "n2", ("g1", "n1"), ("g1", "n2"), ("g2", "n3")]
    for f in W.unpack(fb, fo):
        for d in rng.sample(dests, rng.randint(1, 3)):
            r.add_route(f, d)
            o.add_route(f, d)
    for t in topics[::9]:
        r.add_route(t, "n3")
        o.add_route(t, "n3")
    rc, ro, rs, rd = e.match_routes_batch(tb, to)
    dc, do, dt, dg = e.match_deliveries_batch(tb, to)
    want_r = [(list(rs[ro[t]:ro[t + 1]]), list(rd[ro[t]:ro[t + 1]])) for t in range(len(topics))]
    want_d = [(list(dt[do[t]:do[t] + dc[t]]), list(dg[do[t]:do[t] + dc[t]])) for t in range(len(topics))]
    tagged = r.match_deliveries_many(topics[:400], tagged=True)
    for t in range(400):
        assert tagged[t] == o.match_deliveries(topics[t]), t
    br = Batcher(e, max_topics=2000, deadline_us=300, routes=True)
    bd = Batcher(e, max_topics=1500, deadline_us=300, deliveries=True)
    got_r, got_d = [None] * len(topics), [None] * len(topics)

    def producer(b, got, k):
        for t in range(k, len(topics), 4):
            def cb(status, ids, ds, t=t):
                assert status == 0
                got[t] = (ids, ds)
            b.submit(topics[t], cb)
    ts = [threading.Thread(target=producer, args=(b, g, k)) for b, g in ((br, got_r), (bd, got_d)) for k in range(4)]
    for x in ts:
        x.start()
    for x in ts:
        x.join()
    br.flush()
    bd.flush()
    assert br.stats()["failed_batches"] == 0 and bd.stats()["failed_batches"] == 0
    br.close()
    bd.close()
    for t in range(len(topics)):
        assert got_r[t] == ([int(x) for x in want_r[t][0]], [int(x) for x in want_r[t][1]]), t
        assert got_d[t] == ([int(x) for x in want_d[t][0]], [int(x) for x in want_d[t][1]]), t
    e.close()


def test_batcher_stats_worst_batch_since_last_read(gpu_device):
    """tm_batcher_stats.max_*: the worst single batch's phases since the
    last resetting read (a device batch ran: its device time is there and
    bounds the mean); a plain read leaves the window alone, a resetting one
    starts it again from zero; tm_batcher_get_stats writes only the round-4
    prefix"""
    from emqx_amd.batcher import Batcher
    fb, fo = W.filters(1)
    e = Engine(device=gpu_device)
    e.insert_many(fb, fo)
    e.commit()
    b = Batcher(e, max_topics=512, deadline_us=200)
    tb, to = W.topics(1, n=2000)
    done = []
    for t in W.unpack(tb, to):
        b.submit(bytes(t), lambda st, ids, d: done.append(st))
    b.flush()
    s = b.stats()
    assert len(done) == 2000 and all(x == 0 for x in done)
    assert s["batches"] >= 4
    assert s["max_device_ns"] > 0 and s["max_device_ns"] * s["batches"] >= s["device_ns"]
    assert s["max_sync_ns"] <= s["max_device_ns"]   # a batch's stream wait is inside its device path
    assert b.stats()["max_device_ns"] == s["max_device_ns"]   # a second reader sees the same window
    b.stats(reset_max=True)
    s2 = b.stats()
    assert s2["max_device_ns"] == 0 and s2["max_wait_ns"] == 0 and s2["batches"] == s["batches"]
    import ctypes
    from emqx_amd import _lib as L
    v1 = L.TmBatcherStats()
    v1.max_wait_ns = 12345
    assert e.lib.tm_batcher_get_stats(b.h, ctypes.byref(v1)) == 0
    assert v1.max_wait_ns == 12345 and v1.batches == s["batches"]   # nothing past the v1 prefix written
    b.close()
    e.close()
