"""Sharded mode on CPU: the partition function, and two
gloo ranks running the all-to-all exchange of keyed per-shard lists
(emqx_amd/shard.py) with per-shard O1 results; the merged lists must equal
O1 over the whole filter set, in order.  This also checks that descending
order key = emqx_trie:match/1 order."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_of_partition():
    from emqx_amd import shard
    fs = [b"a/+", b"a/b/#", b"+/x", b"#", b"b/c", b"a", b"+/+/#", b"$SYS/#", b"", b"/a"]
    for s in (1, 2, 3, 8):
        owners = [shard.shard_of(f, s) for f in fs]
        assert all(0 <= x < s for x in owners)
        # one prefix through the 2nd literal level -> one shard
        assert shard.shard_of(b"a/b/+", s) == shard.shard_of(b"a/b/#", s) == shard.shard_of(b"a/b", s)
        assert shard.shard_of(b"+/b/c/d", s) == shard.shard_of(b"+/b/c/+", s) == shard.shard_of(b"+/b/c", s)
        assert shard.shard_of(b"+/+/#", s) == shard.shard_of(b"+/+/#", s)
    # root wildcards and one root's subtrees spread over every shard
    assert np.unique([shard.shard_of(b"+/%d" % i, 8) for i in range(400)]).size == 8
    assert np.unique([shard.shard_of(b"a/%d/#" % i, 8) for i in range(400)]).size == 8
    assert np.unique([shard.shard_of(b"+/+/%d/x" % i, 8) for i in range(400)]).size == 8
    from emqx_amd import workload as W
    fb, fo = W.filters(4, n=200_000)
    load = np.bincount(shard.shard_of_batch(fb, fo, 8), minlength=8) / 25_000
    assert load.max() < 1.6, load


def _workload():
    """C1 filters and topics plus a 32-64-level slice (two-word keys)"""
    from emqx_amd import workload as W
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from long_topics import long_case
    fb, fo = W.filters(1, n=6000)
    tb, to = W.topics(1, n=3000)
    lf, lt = long_case(7, n_filters=800, n_topics=120)
    return W.unpack(fb, fo) + lf, W.unpack(tb, to) + lt


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    from emqx_amd import shard
    from emqx_amd.engine import pack
    from oracle import O1
    from shard_ref import merge_host, order_key
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    filters, topics = _workload()
    mine, seen = [], set()
    for f in filters:
        if shard.shard_of(f, world) == rank and f not in seen:
            seen.add(f)
            mine.append(f)                  # local id = insertion sequence
    o1 = O1()
    fb, fo = pack(mine)
    o1.insert_many(fb, fo)
    tb, to = pack(topics)
    counts, offs, ids = o1.match_ids(tb, to)
    levels = [t.count(b"/") + 1 for t in topics]
    KW = shard.key_words_for(tb, to)
    assert KW == 3
    cap = max(len(ids), 1)
    keys = np.zeros((KW, cap), dtype=np.uint64)
    for t in range(len(topics)):
        for j in range(int(offs[t]), int(offs[t + 1])):
            keys[:, j] = order_key(mine[ids[j]], levels[t], KW)
    rc, base, rid, rk, m = shard.exchange(
        torch.from_numpy(counts.astype(np.int32)), torch.from_numpy(offs.astype(np.int64)),
        torch.from_numpy(ids.astype(np.int32)), torch.from_numpy(keys.reshape(-1).view(np.int64)), len(topics),
        world, rank, key_words=KW, key_stride=cap)
    merged = merge_host(rc.numpy(), base.numpy(), rid.numpy(), rk.numpy(), m, world, key_words=KW)
    # gid -> (shard, local) -> bytes: gather every shard's filter list
    lists = [None] * world
    dist.all_gather_object(lists, mine)
    out = [[lists[g % world][g // world] for g in row] for row in merged]
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_exchange_and_merge_equals_o1():
    from emqx_amd.engine import pack
    from oracle import O1
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    filters, topics = _workload()
    o1 = O1()
    fb, fo = pack(filters)
    o1.insert_many(fb, fo)
    want = [o1.match(t) for t in topics]
    got = res[0] + res[1]
    assert len(got) == len(topics)
    assert sum(len(r) for r in want) > 1000
    assert got == want


def test_wide_order_key_is_reference_order():
    """descending multi-word order key = emqx_trie:match/1 order (O1) for
    topics of 32-64 levels, where groups of filters tie on key word 0"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from emqx_amd.engine import pack
    from long_topics import long_case
    from oracle import O1
    from shard_ref import order_key
    filters, topics = long_case(11)
    o1 = O1()
    o1.insert_many(*pack(filters))
    ties = 0
    for t in topics:
        want = o1.match(t)
        n = t.count(b"/") + 1
        keys = [order_key(f, n, 3) for f in want]
        assert keys == sorted(keys, reverse=True) and len(set(keys)) == len(keys), t
        ties += len(want) - len({k[0] for k in keys})
    assert ties > 100     # word 0 alone would not order them
