"""The routed sharded mode's distributed logic on CPU: two gloo ranks, each
with its own publish batch.  Every topic goes to the rank that owns its first
`depth` levels (tm_route_of, the same function the device routing kernel
computes); that rank holds only its shard's filters (the routed ones and the
wildcard-led ones every shard keeps: the placement tm_insert_batch_routed
makes) and answers with O1, the restatement of emqx_trie:match/1, standing in
for its walk; the lists travel back to the sending rank.  Each rank's lists,
in its own topic order, must equal O1 over the WHOLE filter set."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, depth, q):
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from emqx_amd import shard
    from emqx_amd import workload as W
    from oracle import O1
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    filters = [bytes(x) for x in W.unpack(*W.filters(1))]
    mine = [bytes(x) for x in W.unpack(*W.topics(1, n=3000 + 500 * rank, stream=rank))]
    # this shard's filters
    o1 = O1()
    for f in filters:
        r = shard.filter_route(f, world, depth)
        if r < 0 or r == rank:
            o1.insert(f)
    # topics to their owners (the topic exchange), in each source's order
    out = [[] for _ in range(world)]
    for i, t in enumerate(mine):
        out[shard.topic_route(t, world, depth)].append((i, t))
    got = [None] * world
    dist.all_gather_object(got, out)
    owned = [(src, i, t) for src in range(world) for (i, t) in got[src][rank]]
    # the owner's walk (O1 stands in), lists back to the sources
    back = [[] for _ in range(world)]
    for src, i, t in owned:
        back[src].append((i, o1.match(t)))
    got2 = [None] * world
    dist.all_gather_object(got2, back)
    lists = [None] * len(mine)
    for owner in range(world):
        for i, lst in got2[owner][rank]:
            lists[i] = lst
    full = O1()
    for f in filters:
        full.insert(f)
    ok = all(lists[i] == full.match(t) for i, t in enumerate(mine))
    q.put((rank, ok, len(owned), len(mine)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_routed_lists_equal_full_trie(world):
    """world 2 and 8 (the routed mode's placement and topic routing over the
    driver's 8-rank launch shape, on the CPU)"""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 2, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res)
    assert sum(o for _, _, o, _ in res) == sum(n for _, _, _, n in res)   # every topic walked once
    assert all(0 < o for _, _, o, _ in res)                               # every rank owns topics
