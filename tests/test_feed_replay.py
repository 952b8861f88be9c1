"""The delta feed (erlang/emqx_trie_gpu_feed.erl, mirrored clause for clause
by emqx_amd/feed.py) replays recorded mnesia table events into the engine
through the same C entry points the NIF calls, and ends equal to the
reference's tables:

  * subscribe / unsubscribe through emqx_router (add_trie_route/1,
    del_trie_route/1: src/emqx_router.erl:226-260), which write both tables;
  * a node-down cleanup (emqx_router_helper:cleanup_routes/1,
    src/emqx_router_helper.erl:118-124, 156-160), which deletes route objects
    ONLY: its filters stay in the trie, stale, and emqx_trie:match/1 keeps
    returning them;
  * re-subscribes to stale filters (emqx_trie:insert/1 of an existing filter
    writes nothing, src/emqx_trie.erl:63-65) and their later unsubscribes;
  * a feed that boots mid-stream: it subscribes first and snapshots later, so
    the events between the two are both in the snapshot and replayed.

The events come from oracle/pytrie.py's transcription of emqx_trie /
emqx_router with table-event recording.  On the CPU (host-only engine) the
check is table equality: every #trie_node{} of the reference (edge_count and
topic, via emqx_trie:lookup/1) and every route bag (get_routes/1), which fixes
match/1 and match_routes/1.  The -m gpu twin runs the same sequences and
compares match/1 and match_routes/1 on the device."""
import random

import numpy as np
import pytest

from emqx_amd import Engine
from emqx_amd.emqx_router import _enc
from emqx_amd.engine import pack
from emqx_amd.feed import TrieFeed
from oracle import pytrie

N1, N2, N3 = b"emqx@n1", b"emqx@n2", b"emqx@n3"


def scenario(seed, n_filters=300):
    """a recorded event sequence: (events, model RouteTable, topics to probe,
    stale filters)"""
    rng = random.Random(seed)
    words = [b"a", b"b", b"c", b"$SYS", b"", b"x"]

    def level():
        r = rng.random()
        return b"+" if r < 0.25 else rng.choice(words)

    filters = set()
    while len(filters) < n_filters:
        ws = [level() for _ in range(rng.randint(1, 4))]
        if rng.random() < 0.3:
            ws[-1] = b"#"
        if rng.random() < 0.1:
            ws = [b"$SYS"] + ws
        filters.add(b"/".join(ws))
    filters = sorted(filters)
    literal = [b"a/b", b"a/b/c", b"x", b"$SYS/a"]   # direct routes (emqx_router.erl:223-224)
    ev = []
    rt = pytrie.RouteTable(ev)
    subs = []
    # 1. subscribe: routes to three nodes, some through $share groups
    for f in filters + literal:
        for _ in range(rng.randint(1, 3)):
            node = rng.choice([N1, N2, N3])
            dest = (b"g%d" % rng.randint(0, 2), node) if rng.random() < 0.2 else node
            rt.add_route(f, dest)
            subs.append((f, dest))
    # 2. unsubscribe a third
    for f, d in rng.sample(subs, len(subs) // 3):
        rt.del_route(f, d)
    # 3. n2 goes down: its routes only
    had = {f for f, bag in rt.routes.items()}
    rt.cleanup_routes(N2)
    stale = sorted(f for f in had if f not in rt.routes and pytrie.wildcard(f) and rt.trie.lookup(f))
    # 4. re-subscribe half the stale filters from n1 / n3, add some new ones
    for f in stale[: len(stale) // 2]:
        rt.add_route(f, rng.choice([N1, N3]))
    for k in range(20):
        rt.add_route(b"new/%d/+" % k, N1)
    # 5. unsubscribe some of the re-subscribed ones (the last route: the trie entry goes)
    for f in stale[: len(stale) // 4]:
        for d in list(rt.routes.get(f, [])):
            rt.del_route(f, d)
    topics = set()
    for _ in range(400):
        topics.add(b"/".join(rng.choice(words) for _ in range(rng.randint(1, 5))))
    topics |= {f.replace(b"+", b"a").replace(b"#", b"b") for f in filters[:100]}
    return ev, rt, sorted(topics), stale


def model_nodes(rt):
    """the reference's #trie_node{} records: node_id -> (edge_count, topic)"""
    return {k[1]: (rec[0], rec[1]) for k, rec in rt.trie.trie_node.items() if k[0] == "bin"}


def check_tables(eng, rt):
    nodes = model_nodes(rt)
    for nid, (cnt, topic) in nodes.items():
        assert eng.lookup(nid) == [(cnt, topic)], nid
    assert eng.filter_count == sum(1 for c, t in nodes.values() if t is not None)
    assert eng.node_count == len(nodes) + 1   # + root
    for topic, bag in rt.routes.items():
        got = [eng.dest_bytes(d) for d in eng.get_routes(topic)]
        assert got == [_enc(d) for d in bag], topic
    assert eng.route_count == sum(len(b) for b in rt.routes.values())


def replay(eng, ev, boot_at=0, snap_at=0, snapshot=None):
    """the feed subscribes at event boot_at, snapshots the tables as of event
    snap_at (>= boot_at), then handles every event from boot_at on"""
    feed = TrieFeed(eng)
    if snapshot is not None:
        feed.boot(*snapshot)
    for e in ev[boot_at:]:
        feed.handle(e)
    feed.commit()
    return feed


def snapshot_at(ev, k):
    """ets:tab2list of both tables after the first k events (a table copy
    rebuilt from the event log itself)"""
    nodes, routes = {}, []
    for e in ev[:k]:
        if e[1] == "emqx_trie_node":
            if e[0] == "write":
                nodes[e[2]] = (e[2], e[3], e[4])
            else:
                nodes.pop(e[2], None)
        elif e[0] == "write":
            if (e[2], e[3]) not in routes:
                routes.append((e[2], e[3]))
        else:
            if (e[2], e[3]) in routes:
                routes.remove((e[2], e[3]))
    return list(nodes.values()), routes


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_replay_equals_reference_tables_node_down_included(seed):
    ev, rt, _, stale = scenario(seed)
    assert stale, "the scenario must leave stale filters"
    eng = Engine(device=-1)
    replay(eng, ev)
    check_tables(eng, rt)
    # the stale filters that were not re-subscribed: in the trie, no routes
    for f in stale[len(stale) // 2:]:
        assert eng.lookup(f) == rt.trie.lookup(f) and rt.trie.lookup(f)[0][1] == f
        assert eng.get_routes(f) == []
    eng.close()


@pytest.mark.parametrize("seed", [4, 5])
def test_feed_boot_subscribes_before_snapshot(seed):
    """a feed started mid-stream: subscription at event s, table snapshot at
    event t > s (writes committed in between are seen twice), replay from s"""
    ev, rt, _, _ = scenario(seed)
    rng = random.Random(seed)
    for _ in range(3):
        s = rng.randrange(len(ev))
        t = rng.randrange(s, len(ev) + 1)
        eng = Engine(device=-1)
        replay(eng, ev, boot_at=s, snapshot=snapshot_at(ev, t))
        check_tables(eng, rt)
        eng.close()


def test_snapshot_then_subscribe_loses_writes():
    """the old boot order (snapshot, then subscribe) misses what commits in
    between: the reason the feed subscribes first"""
    ev, rt, _, _ = scenario(6)
    s = len(ev) // 2
    eng = Engine(device=-1)
    replay(eng, ev, boot_at=s + 50, snapshot=snapshot_at(ev, s))   # events s..s+49 lost
    with pytest.raises(AssertionError):
        check_tables(eng, rt)
    eng.close()


def test_route_table_events_never_touch_the_trie():
    eng = Engine(device=-1)
    eng.route_write(b"a/+", b"n1")              # route before its filter: no trie entry
    assert eng.lookup(b"a/+") == [] and eng.filter_count == 0
    eng.insert(b"a/+")                          # the trie event: the route joins the filter
    eng.route_delete_object(b"a/+", b"n1")      # last route gone: the filter stays
    assert eng.lookup(b"a/+") == [(0, b"a/+")]
    eng.route_delete_object(b"a/+", b"n1")      # absent: no-op
    eng.route_write(b"a/+", b"n2")
    eng.delete(b"a/+")                          # the trie event: routes stay in the bag
    assert eng.lookup(b"a/+") == [] and len(eng.get_routes(b"a/+")) == 1
    # the emulating entry points keep del_trie_route/1: the last route takes the filter
    eng.route_add(b"s/#", b"n1")
    eng.route_del(b"s/#", b"n1")
    assert eng.lookup(b"s/#") == []
    eng.close()


def test_whole_key_route_delete_event():
    """mnesia:delete({emqx_route, T}) (not issued by emqx_router, but a
    table operation the feed must follow: erlang/emqx_trie_gpu_feed.erl:97-99)
    arrives as ("delete", "emqx_route", T, Old): every old object goes, the
    trie keeps the filter, other topics' routes stay"""
    eng = Engine(device=-1)
    feed = TrieFeed(eng)
    for e in [("write", "emqx_trie_node", b"a/+", 0, b"a/+"), ("write", "emqx_route", b"a/+", b"n1"),
              ("write", "emqx_route", b"a/+", (b"g1", b"n2")), ("write", "emqx_route", b"b/#", b"n1"),
              ("delete", "emqx_route", b"a/+", [b"n1", (b"g1", b"n2")])]:
        feed.handle(e)
    feed.commit()
    assert eng.get_routes(b"a/+") == [] and eng.lookup(b"a/+") == [(0, b"a/+")]
    assert [eng.dest_bytes(d) for d in eng.get_routes(b"b/#")] == [_enc(b"n1")]
    assert eng.route_count == 1
    eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_replay_match_and_match_routes_node_down(gpu_device, seed):
    """the device twin: match/1 returns the stale filters as emqx_trie:match/1
    does, match_routes/1 equals the reference's (no routes for them)"""
    from emqx_amd.emqx_router import Router
    ev, rt, topics, stale = scenario(seed)
    eng = Engine(device=gpu_device)
    feed = TrieFeed(eng)
    half = len(ev) // 2
    for e in ev[:half]:                         # a batch between the events: epochs flip mid-stream
        feed.handle(e)
    feed.commit()
    buf, off = pack(topics)
    eng.match_batch(buf, off)
    for e in ev[half:]:
        feed.handle(e)
    feed.commit()
    counts, offs, ids = eng.match_batch(buf, off)
    names = eng.filters_bytes(ids)
    k = 0
    for i, t in enumerate(topics):
        got = names[int(offs[i]):int(offs[i + 1])]
        assert got == rt.trie.match(t), t
        k += len(got)
    assert any(f in names for f in stale[len(stale) // 2:]), "no stale filter matched: weak scenario"
    # match_routes/1 over the same engine
    dec = {}
    for e in ev:
        if e[1] == "emqx_route":
            dec[_enc(e[3])] = e[3]
    rc, ro, src, dst = eng.match_routes_batch(buf, off)
    for i, t in enumerate(topics):
        row = []
        for j in range(int(ro[i]), int(ro[i]) + int(rc[i])):
            s = int(src[j])
            to = t if s == Engine.TOPIC_ROUTE else eng.filter_bytes(s)
            row.append((to, dec[eng.dest_bytes(int(dst[j]))]))
        assert row == rt.match_routes(t), t
    eng.close()
