"""Sharded mode on the GPU: S shard engines on one device
(the all-to-all done by slicing, as each rank would receive it), keyed walks
(tm_match_batch_device_keys) and the device merge (tm_shard_merge) must give
emqx_trie:match/1 over the WHOLE filter set, id for id and in order."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

pytestmark = pytest.mark.gpu


def _run_sharded(filters, topics, S, K=None, opts=None):
    import torch
    from emqx_amd import shard
    from emqx_amd.engine import pack
    dev = torch.device("cuda", 0)
    fb, fo = pack(filters)
    tb, to = pack(topics)
    n = len(topics)
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    KW = shard.key_words_for(tb, to)
    engs, res = [], []
    for s in range(S):
        e = shard.ShardEngine(0, S, s, filters_hint=len(filters))
        if K:
            e.set_option("stage_k", K)
        for k, v in (opts or {}).items():
            e.set_option(k, v)
        e.insert_many(fb, fo)
        c = torch.empty(n, dtype=torch.int32, device=dev)
        o = torch.empty(n + 1, dtype=torch.int64, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, None, None, 0, tot, key_words=KW)
        torch.cuda.synchronize()
        cap = int(tot.item()) + 16
        ids = torch.empty(cap, dtype=torch.int32, device=dev)
        keys = torch.empty(cap * KW, dtype=torch.int64, device=dev)
        e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, ids, keys, cap, tot, key_words=KW)
        torch.cuda.synchronize()
        assert e.key_levels() <= 32 * KW - 1
        engs.append(e)
        res.append((c, o, ids, keys.view(KW, cap)))
    b = shard.slices(n, S)
    out = []
    for r in range(S):      # what rank r receives from every shard, then merges
        m = b[r + 1] - b[r]
        rc = torch.cat([res[s][0][b[r]:b[r + 1]] for s in range(S)])
        cuts = [(int(res[s][1][b[r]].item()), int(res[s][1][b[r + 1]].item())) for s in range(S)]
        rid = torch.cat([res[s][2][lo:hi] for s, (lo, hi) in enumerate(cuts)] + [torch.zeros(1, dtype=torch.int32,
                                                                                             device=dev)])
        sizes = [hi - lo for lo, hi in cuts]
        tot_r = sum(sizes)
        # key planes of the received total (what shard.exchange delivers)
        rk = torch.cat([torch.cat([res[s][3][j, lo:hi] for s, (lo, hi) in enumerate(cuts)])
                        for j in range(KW)] + [torch.zeros(1, dtype=torch.int64, device=dev)])
        base = torch.tensor(np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64), device=dev)
        oc = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
        oo = torch.empty(m + 1, dtype=torch.int64, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        cap = sum(sizes) + 1
        og = torch.empty(cap, dtype=torch.int32, device=dev)
        engs[r].merge_device(m, rc, base, rid, rk, oc, oo, og, cap, tot, key_words=KW, key_stride=tot_r)
        torch.cuda.synchronize()
        assert int(tot.item()) == sum(sizes)
        oo_h, og_h = oo.cpu().numpy(), og.cpu().numpy().view(np.uint32)
        for t in range(m):
            out.append([engs[g % S].filter_bytes(int(g) // S) for g in og_h[oo_h[t]:oo_h[t + 1]]])
    for e in engs:
        e.close()
    return out


def _o1(filters, topics):
    from emqx_amd.engine import pack
    from oracle import O1
    o1 = O1(len(filters))
    fb, fo = pack(filters)
    o1.insert_many(fb, fo)
    return [o1.match(t) for t in topics]


@pytest.mark.parametrize("S", [1, 3, 8])
def test_sharded_c1_equals_o1(gpu_device, S):
    from emqx_amd import workload as W
    filters = W.unpack(*W.filters(1))
    topics = W.unpack(*W.topics(1, n=20000))
    got = _run_sharded(filters, topics, S)
    assert got == _o1(filters, topics)


@pytest.mark.parametrize("S,presort", [(1, 1), (3, 1), (3, 2)])
def test_sharded_presorted_walk_equals_o1(gpu_device, S, presort):
    """option presort (1 word-hash key, 2 the tail order) on the keyed walk:
    stage rows in walk order, keys and ids copied out by position
    (tm_copy_out_sorted<KEYS>), merged by key; with a small stage row, so
    topics past K re-walk their heads"""
    from emqx_amd import workload as W
    filters = W.unpack(*W.filters(1))
    topics = W.unpack(*W.topics(1, n=20000))
    got = _run_sharded(filters, topics, S, K=16, opts={"presort": presort, "stage_auto": 0, "shape_keys": 0})
    assert got == _o1(filters, topics)


def test_sharded_shape_keys_with_wave_walk_equal_o1(gpu_device):
    """shape keys over the wave-per-topic walk (small batches)"""
    from emqx_amd import workload as W
    filters = W.unpack(*W.filters(1))
    topics = W.unpack(*W.topics(1, n=5000))
    got = _run_sharded(filters, topics, 3, K=16, opts={"wave_walk_max": 1 << 30})
    assert got == _o1(filters, topics)


@pytest.mark.parametrize("wave", [0, 1])
def test_key_levels_reported_by_every_walk(gpu_device, wave):
    """tm_key_levels after a shaped batch of <= 31-level key width that holds
    a 40-level topic: both the per-lane walk and the wave-per-topic walk
    (small batches) report its 40 levels, so the caller's key-width guard
    (ShardSet.match_batch) fires instead of merging with truncated keys"""
    import torch
    from emqx_amd import shard
    from emqx_amd.engine import pack
    dev = torch.device("cuda", 0)
    long_t = b"/".join(b"l%d" % i for i in range(40))
    filters = [b"l0/#", b"+/l1/#", b"#", long_t, b"a/+"]
    topics = [b"a/b", long_t, b"x/y/z"] * 20
    fb, fo = pack(filters)
    tb, to = pack(topics)
    n = len(topics)
    e = shard.ShardEngine(0, 1, 0, filters_hint=len(filters))
    e.set_option("wave_walk_max", (1 << 30) if wave else 0)
    e.insert_many(fb, fo)
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)
    o = torch.empty(n + 1, dtype=torch.int64, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, None, None, 0, tot, key_words=1)
    torch.cuda.synchronize()
    cap = int(tot.item()) + 16
    ids = torch.empty(cap, dtype=torch.int32, device=dev)
    keys = torch.empty(cap, dtype=torch.int64, device=dev)
    e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, ids, keys, cap, tot, key_words=1)   # the keyed batch
    torch.cuda.synchronize()
    assert e.key_levels() == 40
    assert shard.key_words_for(tb, to) == 2   # what ShardSet would have chosen
    e.close()


@pytest.mark.parametrize("shape", [0, 1])
def test_sharded_walk_keys_and_shape_keys_equal_o1(gpu_device, shape):
    """both ways to key a shard's lists: the keyed walk (rank_sym) and the
    unkeyed walk whose copy-out takes each filter's order key
    (image.h filter_shape, option shape_keys, the ShardEngine default)"""
    from emqx_amd import workload as W
    filters = W.unpack(*W.filters(2, n=200_000))
    topics = W.unpack(*W.topics(2, n=20000))
    got = _run_sharded(filters, topics, 3, opts={"shape_keys": shape})
    assert got == _o1(filters, topics)


@pytest.mark.parametrize("S", [1, 3])
def test_sharded_out_of_domain_topic_levels_equal_o1(gpu_device, S):
    """publish topics with literal '+' / '#' levels (rejected by
    emqx_packet.erl:63, so out of the domain, but emqx_trie:match/1 still
    answers them: the fold over [W, '+'] follows the '+' edge twice and the
    list repeats filters).  With shape keys such a topic's lists are keyed by
    a keyed re-walk in the copy-out (filter keys would tie)"""
    import random
    rng = random.Random(5)
    words = [b"a", b"b", b"+", b"#", b""]
    filters = set()
    while len(filters) < 1500:   # of ~4,700 possible
        ws = [rng.choice([b"a", b"b", b"c", b"+", b""]) for _ in range(rng.randint(1, 5))]
        if rng.random() < 0.3:
            ws[-1] = b"#"
        filters.add(b"/".join(ws))
    filters = sorted(filters)
    topics = [b"/".join(rng.choice(words) for _ in range(rng.randint(1, 5))) for _ in range(3000)]
    assert sum(1 for t in topics if b"+" in t.split(b"/") or b"#" in t.split(b"/")) > 500
    got = _run_sharded(filters, topics, S, K=8)
    assert got == _o1(filters, topics)


def test_sharded_c5_sample_equals_o1(gpu_device):
    """16-level '#'-heavy topics, $SYS, $share via parse, fan-out > K (re-walk with keys)"""
    from emqx_amd import emqx_topic as T
    from emqx_amd import workload as W
    filters = [T.parse(f)[0] for f in W.unpack(*W.filters(5, n=100_000))]
    topics = W.unpack(*W.topics(5, n=1500))
    want = _o1(filters, topics)
    assert max(len(r) for r in want) > 512
    got = _run_sharded(filters, topics, 4, K=256)
    assert got == want


def test_sharded_kats(gpu_device, golden):
    """the reference's own trie KATs and the O1 vectors, split over 3 shards"""
    for vec in golden["o1_vectors"]:
        topics = [r["topic"].encode("latin-1") for r in vec["topics"]]
        filters = [f.encode("latin-1") for f in vec["filters"]]
        got = _run_sharded(filters, topics, 3)
        assert [[x.decode("latin-1") for x in row] for row in got] == [r["match"] for r in vec["topics"]], vec["name"]


def test_sharded_topic_beyond_lds_merge(gpu_device):
    """a topic with > 1024 matches (all 2^11 literal/'+' combinations of an
    11-level topic, plus '#' prefixes) takes the merge's serial path"""
    import itertools
    words = [b"l%d" % i for i in range(11)]
    filters = [b"/".join(w if bit else b"+" for w, bit in zip(words, bits))
               for bits in itertools.product([0, 1], repeat=11)]
    filters += [b"/".join(words[:k] + [b"#"]) for k in range(11)]
    topics = [b"/".join(words), b"l0/l1/x", b"/".join(words[:5]), b"$SYS/l1"]
    want = _o1(filters, topics)
    assert len(want[0]) > 1024
    for S in (2, 5):
        assert _run_sharded(filters, topics, S, K=256) == want


@pytest.mark.parametrize("S", [3, 8])
def test_sharded_32_to_64_levels_equals_o1(gpu_device, S):
    """keys of 2+ words; topics of 32-64 levels, id for id vs O1"""
    from emqx_amd import shard
    from emqx_amd.engine import pack
    from long_topics import long_case
    filters, topics = long_case(S)
    tb, to = pack(topics)
    assert shard.key_words_for(tb, to) == 3
    want = _o1(filters, topics)
    assert sum(len(w) for w in want) > 1000 and max(len(w) for w in want) > 8
    assert _run_sharded(filters, topics, S) == want
    assert _run_sharded(filters, topics, S, K=4) == want   # re-walk tail with wide keys


@pytest.mark.parametrize("S", [2, 3])
def test_shardset_native_exchange_equals_o1(gpu_device, S):
    """all shards of one process through the C-ABI exchange
    (tm_comm_init_all + tm_shard_exchange_group; the shards share GPU 0, so
    it moves the lists by device copies) and the device merge"""
    from emqx_amd import shard
    from emqx_amd import workload as W
    from emqx_amd.engine import pack
    from long_topics import long_case
    filters = W.unpack(*W.filters(1))
    topics = W.unpack(*W.topics(1, n=8000))
    lf, lt = long_case(5, n_filters=600, n_topics=100)
    filters, topics = filters + lf, topics + lt
    fb, fo = pack(filters)
    tb, to = pack(topics)
    ss = shard.ShardSet([gpu_device] * S)
    assert not any(c.rccl for c in ss.comms)
    ss.insert_many(fb, fo)
    counts, offs, gids = ss.match_batch(tb, to)
    want = _o1(filters, topics)
    got = [[ss.filter_bytes(int(g)) for g in gids[offs[t]:offs[t + 1]]] for t in range(len(topics))]
    assert got == want
    ss.close()


@pytest.mark.parametrize("self_rccl", [False, True])
def test_rccl_one_rank_exchange_equals_o1(gpu_device, self_rccl):
    """the RCCL path of tm_shard_exchange on the one GPU of the box: a
    one-rank communicator (the size all-to-all over RCCL; with self_rccl the
    counts, ids and keys too, by send / receive to itself inside the group),
    then the merge"""
    import torch
    from emqx_amd import shard
    from emqx_amd import workload as W
    from emqx_amd.engine import pack
    filters = W.unpack(*W.filters(1))
    topics = W.unpack(*W.topics(1, n=5000))
    fb, fo = pack(filters)
    tb, to = pack(topics)
    comm = shard.Comm.init_rank(shard.Comm.unique_id(), 1, 0, gpu_device)
    assert comm.rccl
    if self_rccl:
        comm.set_self_rccl(True)
    e = shard.ShardEngine(gpu_device, 1, 0)
    e.insert_many(fb, fo)
    dev = torch.device("cuda", gpu_device)
    n = len(topics)
    d_b = torch.from_numpy(tb.copy()).to(dev)
    d_o = torch.from_numpy(to.view(np.int64).copy()).to(dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)
    o = torch.empty(n + 1, dtype=torch.int64, device=dev)
    t = torch.zeros(1, dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(device=dev)   # one explicit stream: walk -> RCCL exchange -> merge
    e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, None, None, 0, t, stream=st)
    st.synchronize()
    cap = int(t.item()) + 1
    ids = torch.empty(cap, dtype=torch.int32, device=dev)
    keys = torch.empty(cap, dtype=torch.int64, device=dev)
    e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, ids, keys, cap, t, stream=st)
    x = shard.exchange_native(comm, c, o, ids, keys, n, key_words=1, key_stride=cap, stream=st)
    assert x.m == n and x.total == cap - 1
    oc = torch.empty(n, dtype=torch.int32, device=dev)
    oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    og = torch.empty(cap, dtype=torch.int32, device=dev)
    e.merge_device(n, x.d_counts, x.d_src_base, x.d_ids, x.d_keys, oc, oo, og, cap, tot, stream=st,
                   key_words=1, key_stride=x.total)
    torch.cuda.synchronize()
    from oracle import O1
    o1 = O1()
    o1.insert_many(fb, fo)
    wc, wo, wi = o1.match_ids(tb, to, threads=4)
    assert np.array_equal(oo.cpu().numpy().view(np.uint64), wo)
    assert np.array_equal(og[: int(wo[-1])].cpu().numpy().view(np.uint32), wi)
    comm.close()
    e.close()


@pytest.mark.parametrize("S,depth", [(4, 2), (8, 1)])
def test_routed_shards_on_device_equal_o1(gpu_device, S, depth):
    """topic routing by first words (shard.py routed_partition): each shard
    engine holds its literal-led filters plus every wildcard-led one and
    walks only the topics it owns; its device lists equal O1 over the whole
    filter set, filter for filter and in order"""
    from emqx_amd import shard
    from emqx_amd import workload as W
    from emqx_amd.engine import Engine
    from oracle import O1
    fb, fo = W.filters(1)
    tb, to = W.topics(1, n=20000)
    filters = [bytes(x) for x in W.unpack(fb, fo)]
    topics = [bytes(x) for x in W.unpack(tb, to)]
    full = O1()
    full.insert_many(fb, fo)
    per, owner, _ = shard.routed_partition(filters, topics, S, depth)
    for s in range(S):
        mine = [t for t, o in zip(topics, owner) if o == s]
        if not mine:
            continue
        e = Engine(device=gpu_device)
        for f in per[s]:
            e.insert(f)
        got = e.match(mine)
        for t, g in zip(mine, got):
            assert list(g) == full.match(t), (s, t)
        e.close()
