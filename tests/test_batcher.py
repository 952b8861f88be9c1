"""Micro-batcher plumbing on CPU (tm_batcher_*): a host-only engine cannot
match, so every submitted topic must complete with TM_EDEVICE (the match
path fails loudly, no CPU fallback); sealing by size and by deadline; flush
and close with requests in flight."""
import threading
import time

from emqx_amd import Engine, _lib
from emqx_amd.batcher import Batcher


def test_batcher_fails_loudly_without_gpu_and_seals():
    e = Engine(device=-1)
    e.insert(b"a/+")
    b = Batcher(e, max_topics=100, deadline_us=300)
    got = []
    lock = threading.Lock()

    def cb(status, ids, dests):
        with lock:
            got.append((status, ids))

    def producer(k):
        for i in range(250):
            b.submit(b"a/%d" % (k * 1000 + i), cb)
    ts = [threading.Thread(target=producer, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    b.flush()
    assert len(got) == 1000
    assert all(s == _lib.TM_EDEVICE and ids is None for s, ids in got)
    st = b.stats()
    assert st["topics"] == 1000 and st["failed_batches"] == st["batches"]
    # a seal takes everything pending, so a batch may pass max_topics by what
    # arrived while it was being sealed
    assert st["size_seals"] + st["deadline_seals"] == st["batches"]
    assert st["size_seals"] >= 1
    b.submit(b"x", cb)           # a lone topic is sealed by the deadline, no flush
    for _ in range(200):
        if len(got) == 1001:
            break
        time.sleep(0.01)
    assert len(got) == 1001 and b.stats()["deadline_seals"] >= 1
    b.close()
    e.close()


def test_callback_threads_complete_every_topic_once():
    """callback threads take parts of a batch (>= 8192 topics each): every
    topic still completes exactly once, before flush returns"""
    e = Engine(device=-1)
    b = Batcher(e, max_topics=40000, deadline_us=2000, callback_threads=3)
    seen = {}
    lock = threading.Lock()

    def producer(k):
        for i in range(20000):
            t = k * 100000 + i

            def cb(status, ids, dests, t=t):
                with lock:
                    seen[t] = seen.get(t, 0) + 1
            b.submit(b"a/%d" % t, cb)
    ts = [threading.Thread(target=producer, args=(k,)) for k in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    b.flush()
    assert len(seen) == 80000 and set(seen.values()) == {1}
    st = b.stats()
    assert st["topics"] == 80000
    b.close()
    e.close()


def test_backlog_partial_takes_complete_every_topic_once():
    """producers far ahead of small batches: seals take a stripe's oldest
    topics and leave the rest (head advance + compaction); every topic still
    completes exactly once and each producer's topics complete in order"""
    e = Engine(device=-1)
    b = Batcher(e, max_topics=64, deadline_us=50, lanes_per_replica=1)
    order = {}
    lock = threading.Lock()

    def producer(k):
        for i in range(5000):
            def cb(status, ids, dests, k=k, i=i):
                with lock:
                    order.setdefault(k, []).append(i)
            b.submit(b"p/%d/%d" % (k, i), cb)
    ts = [threading.Thread(target=producer, args=(k,)) for k in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    b.flush()
    assert sorted(order) == [0, 1, 2]
    for k in range(3):   # one lane: batches complete in seal order, a stripe's topics oldest first
        assert order[k] == list(range(5000)), k
    b.close()
    e.close()
