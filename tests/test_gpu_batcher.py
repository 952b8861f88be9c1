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


@pytest.mark.parametrize("routes", [False, True, "deliveries"])
def test_batcher_results_equal_batch_api(gpu_device, routes):
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
    b = Batcher(e, max_topics=3000, deadline_us=500, routes=routes is True, deliveries=routes == "deliveries")
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
    assert st["topics"] == len(topics) and st["failed_batches"] == 0 and st["batches"] >= 5
    for t in range(len(topics)):
        ids, dests = got[t]
        assert [int(x) for x in want[t][0]] == ids, t
        if routes:
            assert [int(x) for x in want[t][1]] == dests, t
    assert sum(len(g[0]) for g in got) > 100_000
    e.close()
