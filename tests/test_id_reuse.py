"""Deferred filter id reuse (engine.cpp quarantine + tm_lease_*).

A match returns filter ids of the image epoch it ran on; the NIF turns them
into binaries afterwards.  If a delete freed an id and an insert took it at
once, those ids would name another filter's bytes (a misrouted delivery), or
the gather would fail for the whole list.  The engine therefore keeps a
deleted filter's id (and its bytes) until both image epochs have dropped it
and no lease older than the deletion's commit is open.  Host-only here; the
-m gpu test churns the trie under running batcher callbacks."""
import random
import threading

import pytest

from emqx_amd import Engine
from oracle import pytrie


def fid(eng, f):
    [(cnt, t)] = eng.lookup(f)
    assert t == f
    import ctypes
    from emqx_amd import _lib as L
    info = L.TmNodeInfo()
    assert eng.lib.tm_lookup(eng.h, f, len(f), ctypes.byref(info)) == 0
    return info.filter_id


def test_deleted_id_keeps_its_bytes_until_two_commits():
    eng = Engine(device=-1)
    eng.insert(b"a/+")
    eng.commit()
    x = fid(eng, b"a/+")
    eng.delete(b"a/+")
    assert eng.filters_bytes([x]) == [b"a/+"]          # still served
    eng.insert(b"b/#")
    assert fid(eng, b"b/#") != x                        # not reused before any commit
    eng.commit()                                        # one image has dropped it
    eng.insert(b"c/+")
    assert fid(eng, b"c/+") != x
    eng.commit()                                        # both have
    eng.insert(b"d/+")
    assert fid(eng, b"d/+") == x                        # now reusable
    assert eng.filters_bytes([x]) == [b"d/+"]
    eng.close()


def test_open_lease_blocks_reuse():
    eng = Engine(device=-1)
    eng.insert(b"a/+")
    eng.commit()
    x = fid(eng, b"a/+")
    with eng.lease():                                   # a reader that may still hold x
        eng.delete(b"a/+")
        for k in range(4):
            eng.commit()
            eng.insert(b"n/%d/+" % k)
            assert fid(eng, b"n/%d/+" % k) != x
            assert eng.filters_bytes([x]) == [b"a/+"]
    eng.commit()
    eng.insert(b"z/+")
    assert fid(eng, b"z/+") == x                        # released with the lease
    eng.close()


def test_lease_taken_after_the_deleting_commit_does_not_block():
    eng = Engine(device=-1)
    eng.insert(b"a/+")
    eng.commit()
    x = fid(eng, b"a/+")
    eng.delete(b"a/+")
    eng.commit()                                        # the deletion is published
    with eng.lease():                                   # this reader can never see x
        eng.commit()
        eng.insert(b"q/+")
        assert fid(eng, b"q/+") == x
    eng.close()


@pytest.mark.gpu
def test_gpu_batcher_callbacks_under_delete_reinsert_churn(gpu_device):
    """batcher callbacks resolve their ids to names while another thread
    deletes and re-inserts filters (ids freed and retaken): every name a
    callback receives must be a filter that matches its topic
    (emqx_topic:match/2), and the never-churned matches must all be there"""
    from emqx_amd.batcher import Batcher
    rng = random.Random(7)
    stable = [b"s/+/%d" % k for k in range(50)] + [b"s/#"]
    churn = [b"s/%d/+" % k for k in range(200)] + [b"zz/%d/#" % k for k in range(400)]
    eng = Engine(device=gpu_device)
    for f in stable + churn:
        eng.insert(f)
    eng.commit()
    topics = [b"s/%d/%d" % (rng.randrange(200), rng.randrange(50)) for _ in range(20000)]
    stop = threading.Event()

    def churner():
        r = random.Random(1)
        live = set(churn)
        while not stop.is_set():
            for f in r.sample(churn, 40):
                if f in live:
                    eng.delete(f)
                    live.discard(f)
                else:
                    eng.insert(f)
                    live.add(f)
            eng.commit()
    th = threading.Thread(target=churner)
    th.start()
    bad, missing, failed = [], [], []
    try:
        b = Batcher(eng, max_topics=4096, deadline_us=200)
        for rnd in range(3):
            def cb_for(t):
                def cb(status, ids, dests):
                    if status != 0:
                        failed.append(status)
                        return
                    names = eng.filters_bytes(ids)   # inside the callback, as the NIF gathers
                    for n in names:
                        if not pytrie.match(t, n):
                            bad.append((t, n))
                    if not set(f for f in stable if pytrie.match(t, f)) <= set(names):
                        missing.append(t)
                return cb
            for t in topics:
                b.submit(t, cb_for(t))
            b.flush()
        b.close()
    finally:
        stop.set()
        th.join()
    assert not failed, failed[:5]
    assert not missing, missing[:5]
    assert not bad, bad[:5]
    eng.close()
