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


# ---- caller-chosen (global) ids: tm_insert_batch_ids (sharded / routed engines)

def _ins_ids(eng, filters, ids):
    from emqx_amd.engine import pack
    b, o = pack(filters)
    eng.insert_many_ids(b, o, ids)


def test_forced_id_of_another_filter_waits_out_the_quarantine():
    """a deleted id taken at once by a forced insert skipped the
    epoch / lease guard.  Now another filter gets it only once both images
    dropped it and no older lease is open; the same filter may take it back
    at once (whatever a batch in flight names, it is still that filter)."""
    from emqx_amd import _lib as L
    eng = Engine(device=-1)
    _ins_ids(eng, [b"a/+", b"b/#"], [7, 9])
    eng.commit()
    assert fid(eng, b"a/+") == 7 and fid(eng, b"b/#") == 9
    eng.delete(b"a/+")
    with pytest.raises(L.TopicMatchError):
        _ins_ids(eng, [b"z/+"], [7])                      # another filter, before any commit
    eng.commit()
    with pytest.raises(L.TopicMatchError):
        _ins_ids(eng, [b"z/+"], [7])                      # one image still holds 7
    assert eng.filters_bytes([7]) == [b"a/+"]
    eng.commit()
    _ins_ids(eng, [b"z/+"], [7])                          # both images dropped it, no lease: reusable
    assert fid(eng, b"z/+") == 7 and eng.filters_bytes([7]) == [b"z/+"]
    # the same filter back under its own id: at once
    eng.delete(b"b/#")
    _ins_ids(eng, [b"b/#"], [9])
    assert fid(eng, b"b/#") == 9
    eng.close()


def test_forced_id_respects_open_leases():
    from emqx_amd import _lib as L
    eng = Engine(device=-1)
    _ins_ids(eng, [b"a/+"], [3])
    eng.commit()
    lease = eng.lease()
    lease.__enter__()
    eng.delete(b"a/+")
    for _ in range(3):
        eng.commit()
        with pytest.raises(L.TopicMatchError):
            _ins_ids(eng, [b"q/+"], [3])
    lease.__exit__(None, None, None)
    eng.commit()
    _ins_ids(eng, [b"q/+"], [3])
    assert fid(eng, b"q/+") == 3
    eng.close()


def test_forced_ids_duplicate_filter_and_live_id():
    """a filter already present under another id was silently
    kept under the old id; a live id is refused as before"""
    from emqx_amd import _lib as L
    eng = Engine(device=-1)
    _ins_ids(eng, [b"s/+/x"], [5])
    _ins_ids(eng, [b"s/+/x"], [5])                        # same filter, same id: idempotent
    with pytest.raises(L.TopicMatchError):
        _ins_ids(eng, [b"s/+/x"], [6])                    # same filter, another id
    with pytest.raises(L.TopicMatchError):
        _ins_ids(eng, [b"t/#"], [5])                      # another filter, a live id
    assert eng.filter_count == 1 and fid(eng, b"s/+/x") == 5
    eng.close()


def test_forced_id_batch_refused_whole():
    """a batch with one refused entry used to leave the entries
    before it inserted (callers have no rollback).  The batch is now checked
    whole first: any bad entry -- a live id, a filter under another id, an id
    or a filter twice in the batch -- refuses it and changes nothing."""
    from emqx_amd import _lib as L
    eng = Engine(device=-1)
    _ins_ids(eng, [b"s/+/x"], [5])
    bad = [
        ([b"a/1", b"b/+", b"t/#"], [10, 11, 5]),          # the last takes a live id
        ([b"a/1", b"s/+/x"], [10, 12]),                   # a present filter under another id
        ([b"a/1", b"b/+"], [10, 10]),                     # one id for two filters
        ([b"a/1", b"a/1"], [10, 13]),                     # one filter under two ids
    ]
    for fl, ids in bad:
        with pytest.raises(L.TopicMatchError):
            _ins_ids(eng, fl, ids)
        assert eng.filter_count == 1 and not eng.lookup(b"a/1") and not eng.lookup(b"b/+"), (fl, ids)
    _ins_ids(eng, [b"a/1", b"a/1", b"s/+/x"], [10, 10, 5])   # repeats with the same partner: fine
    assert eng.filter_count == 2 and fid(eng, b"a/1") == 10
    eng.close()


def test_forced_only_engine_drains_its_quarantine_at_commit():
    """a forced-only engine (routed shards) never calls the id allocator, so
    the quarantine must drain at commit: many delete / re-insert rounds of
    distinct filters under recycled ids all succeed after two commits"""
    eng = Engine(device=-1)
    ids = list(range(100, 164))
    _ins_ids(eng, [b"r0/%d/+" % i for i in ids], ids)
    eng.commit()
    for rnd in range(1, 6):
        for i in ids:
            eng.delete(b"r%d/%d/+" % (rnd - 1, i))
        eng.commit()
        eng.commit()
        _ins_ids(eng, [b"r%d/%d/+" % (rnd, i) for i in ids], ids)
        assert all(fid(eng, b"r%d/%d/+" % (rnd, i)) == i for i in ids)
    eng.close()


def test_routed_insert_repeated_filter_keeps_first_id():
    """tm_insert_batch_routed over a list with repeats: emqx_trie:insert/1 is
    idempotent, so the repeat keeps its first index (a list's filter i is
    named by the first i holding it)"""
    from emqx_amd import shard
    from emqx_amd.engine import pack
    eng = shard.RoutedEngine(-1, 1, 0, depth=1)
    b, o = pack([b"x/+", b"y/#", b"x/+", b"z"])
    eng.insert_many(b, o)
    assert fid(eng, b"x/+") == 0 and fid(eng, b"y/#") == 1 and fid(eng, b"z") == 3
    assert eng.filter_count == 3
    eng.close()
