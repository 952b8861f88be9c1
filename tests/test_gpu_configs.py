"""SURVEY §8(d) configurations at their full filter counts on the GPU
(VERDICT r1 "untested configs"):

* C3 — 10M filters, a 100K-topic sample id for id against O1, whole and
  split 2/4/8 ways (the strong-scaling split bench.py uses per rank);
* C5 — all 1M adversarial filters ($share via parse, '#'-heavy, 16 levels,
  fan-out ~900), 10K topics against O1;
* C4 — 100M filters sharded over S = 8 shard engines emulated on one GPU
  (keyed walks, the exchange as each rank would receive it, device merge):
  a 20K-topic sample of the merged lists against the replicated whole-set
  engine (itself O1-pinned at C3).

Long steps print a progress line (capture disabled), so a slow build never
looks like a hang."""
import os
import sys
import threading
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


class _Progress:
    def __init__(self, capsys, name):
        self.capsys, self.name, self.t0 = capsys, name, time.time()

    def __call__(self, msg):
        with self.capsys.disabled():
            print("[%s %5.0fs] %s" % (self.name, time.time() - self.t0, msg), flush=True)


def _threads(*fns):
    """run fns in threads (the C calls release the GIL), re-raise failures"""
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as x:   # noqa: BLE001
            errs.append(x)
    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def _threads_for_o1():
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count())


def test_c3_10m_filters_100k_topics_vs_o1(gpu_device, capsys):
    from emqx_amd import Engine, multi
    from emqx_amd import workload as W
    from oracle import O1
    say = _Progress(capsys, "C3")
    fb, fo = W.filters(3)
    tb, to = W.topics(3, n=100_000)
    say("generated 10M filters, 100K topics")
    box = {}

    def build_engine():
        e = Engine(device=gpu_device, filters_hint=10_000_000)
        e.insert_many(fb, fo)
        e.commit()
        box["e"] = e

    def build_o1():
        o = O1(10_000_000)
        o.insert_many(fb, fo)
        box["o"] = o
    _threads(build_engine, build_o1)
    e, o1 = box["e"], box["o"]
    assert e.filter_count == 10_000_000
    say("engine + O1 built: %d nodes" % e.node_count)
    oc, oo, oi = o1.match_ids(tb, to, threads=_threads_for_o1())
    counts, offs, ids = e.match_batch(tb, to)
    assert np.array_equal(counts, oc) and np.array_equal(offs, oo) and np.array_equal(ids, oi)
    assert oo[-1] > 50 * 100_000     # C3 fan-out ~56
    say("100K topics bit-exact, %d matches" % int(oo[-1]))
    n = len(to) - 1
    for world in (2, 4, 8):          # the batch split the way bench.py splits it over ranks
        for rank in range(world):
            lo, hi = multi.batch_slice(n, world, rank)
            sub = (to[lo:hi + 1] - to[lo]).astype(np.uint64)
            c, of, i = e.match_batch(tb[int(to[lo]):int(to[hi]) + 8], sub)
            assert np.array_equal(c, oc[lo:hi])
            assert np.array_equal(i, oi[int(oo[lo]):int(oo[hi])])
    say("2/4/8-way splits bit-exact")
    e.close()


def test_c5_1m_filters_vs_o1(gpu_device, capsys):
    from emqx_amd import Engine
    from emqx_amd import emqx_topic as T
    from emqx_amd import workload as W
    from emqx_amd.engine import pack
    from oracle import O1
    say = _Progress(capsys, "C5")
    raw = W.unpack(*W.filters(5))
    inner = [T.parse(f)[0] for f in raw]        # $share/g/F -> F (emqx_topic:parse/1)
    assert sum(1 for f in raw if f.startswith(b"$share/")) > 50_000
    fb, fo = pack(inner)
    tb, to = W.topics(5, n=10_000)
    box = {}

    def build_engine():
        e = Engine(device=gpu_device, filters_hint=1_000_000)
        e.insert_many(fb, fo)
        e.commit()
        box["e"] = e

    def build_o1():
        o = O1(1_000_000)
        o.insert_many(fb, fo)
        box["o"] = o
    _threads(build_engine, build_o1)
    e, o1 = box["e"], box["o"]
    say("built: %d filters (after $share collapse), %d nodes" % (e.filter_count, e.node_count))
    oc, oo, oi = o1.match_ids(tb, to, threads=_threads_for_o1())
    counts, offs, ids = e.match_batch(tb, to)
    assert np.array_equal(counts, oc) and np.array_equal(offs, oo) and np.array_equal(ids, oi)
    assert oc.mean() > 500 and oc.max() > 1000
    say("10K topics bit-exact, mean fan-out %.0f, max %d" % (oc.mean(), oc.max()))
    e.close()


def test_c4_100m_filters_sharded_8_vs_replicated_vs_o3(gpu_device, capsys):
    from emqx_amd import Engine, shard
    from emqx_amd import workload as W
    say = _Progress(capsys, "C4")
    S = 8
    fb, fo = W.filters(4)
    n_f = len(fo) - 1
    assert n_f == 100_000_000
    say("generated 100M filters (%.1f GB)" % (fo[-1] / 1e9))
    engs = [None] * S
    box = {}

    def build_rep():
        e = Engine(device=gpu_device, filters_hint=n_f)
        # the whole-set reference side keeps insertion order (no relayout of
        # its 252M nodes: the long pole of this test); layout variants are
        # parity-tested against O1 in test_gpu_parity.py
        e.set_option("layout", 0)
        e.insert_many(fb, fo)
        e.commit()
        box["rep"] = e

    def build_o3():
        # the oracle side: O3 (oracle/o3_interned.c, emqx_trie's algorithm over
        # interned ids) over all 100M filters
        from oracle import O3
        o = O3(n_f)
        o.insert_many(fb, fo)
        box["o3"] = o

    def build_shard(s):
        e = shard.ShardEngine(gpu_device, S, s, filters_hint=n_f // S + 1)
        e.set_option("stage_k", 128)
        e.insert_many(fb, fo)
        e.commit()
        engs[s] = e

    done = threading.Event()

    def ticker():
        while not done.wait(30):
            say("building 9 engines ...")
    tk = threading.Thread(target=ticker)
    tk.start()
    try:
        _threads(build_rep, build_o3, *[(lambda s=s: build_shard(s)) for s in range(S)])
    finally:
        done.set()
        tk.join()
    rep = box["rep"]
    assert rep.filter_count == n_f and sum(x.filter_count for x in engs) == n_f
    say("built: replicated %d nodes, shards %s filters" % (rep.node_count, [x.filter_count for x in engs]))
    tb, to = W.topics(4, n=20_000)
    n = len(to) - 1
    # the product path of the sharded mode in one process: every shard's keyed
    # walk, tm_shard_exchange_group (the 8 shards share this GPU, so the
    # exchange moves each slice by device copies where ranks on 8 GPUs use
    # RCCL), then each slice's device merge (shard.ShardSet.match_batch)
    ss = shard.ShardSet([gpu_device] * S, engines=engs)
    assert not any(c.rccl for c in ss.comms)
    m_counts, m_offs, m_gids = ss.match_batch(tb, to)
    merged_off = m_offs
    merged_gid = [m_gids]
    say("sharded walk + exchange (tm_shard_exchange_group) + merge done")
    counts, offs, ids = rep.match_batch(tb, to)
    assert np.array_equal(m_counts, counts)
    assert np.array_equal(np.asarray(merged_off, dtype=np.uint64), offs)
    # both id spaces -> the filter's index in the generated list: the
    # replicated engine numbers distinct filters in insertion order, a shard
    # gid is local * S + shard
    g2i = shard.gid_to_index(shard.shard_of_batch(fb, fo, S), S)
    got = g2i[np.concatenate(merged_gid).astype(np.int64)]
    assert np.array_equal(got, ids.astype(np.int64))
    assert offs[-1] > 60 * n
    say("20K topics: sharded (S=8) == replicated, %d matches" % int(offs[-1]))
    # pinned to the oracle: O3's ordered lists of the first 10K topics equal
    # the replicated engine's (and so the sharded merge's), id for id
    k = 10_000
    oc, oo, oi = box["o3"].match_ids(tb, to[: k + 1], threads=8)
    assert np.array_equal(oc, counts[:k]) and np.array_equal(oo, offs[: k + 1])
    assert np.array_equal(oi, ids[: int(oo[-1])])
    say("10K topics: replicated == O3 over 100M filters, %d matches" % int(oo[-1]))
    box["o3"].close()
    ss.close()
    rep.close()
