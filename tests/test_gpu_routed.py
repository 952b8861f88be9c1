"""Routed sharded mode on the GPU (topicmatch.h tm_route_*):
S routed shard engines sharing GPU 0 in one process (tm_route_exchange_group
/ tm_route_return_group move the topics and lists by device copies, the RCCL
path's same transfers).  Every rank hands in its own publish batch; each
topic is walked only on the shard that owns its first `depth` levels, and the
lists come back to the rank that sent it.  They must equal emqx_trie:match/1
over the WHOLE filter set (O1), id for id (global ids = the filter's index)
and in order, on every rank."""
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu
L1 = "latin-1"


def _run(filters_b, filters_o, batches, S, depth):
    from emqx_amd import shard
    rs = shard.RoutedSet([0] * S, depth=depth, filters_hint=len(filters_o))
    try:
        rs.insert_many(filters_b, filters_o)
        return rs.match_batches(batches)
    finally:
        rs.close()


def _check(fb, fo, batches, got):
    from oracle import O1
    o1 = O1(len(fo))
    o1.insert_many(fb, fo)
    for r, ((tb, to), (c, oo, ids)) in enumerate(zip(batches, got)):
        oc, ooo, oi = o1.match_ids(tb, to, threads=8)
        assert np.array_equal(c, oc), r
        assert np.array_equal(oo, ooo), r
        if not np.array_equal(ids, oi):   # name the first topic whose list differs
            j = int(np.flatnonzero(ids != oi)[0])
            t = int(np.searchsorted(ooo, j, side="right")) - 1
            bad = [int(x) for x in np.flatnonzero([not np.array_equal(ids[ooo[u]:ooo[u + 1]], oi[ooo[u]:ooo[u + 1]])
                                                   for u in range(len(oc))])]
            raise AssertionError(f"rank {r}: {len(bad)} topics differ, first {t} "
                                 f"{bytes(tb[to[t]:to[t + 1]])!r}: got {ids[ooo[t]:ooo[t + 1]].tolist()} "
                                 f"want {oi[ooo[t]:ooo[t + 1]].tolist()}; topics {bad[:20]}")
    o1.close()


@pytest.mark.parametrize("S,depth", [(2, 1), (3, 2), (4, 2)])
def test_routed_c1_every_rank_equals_o1(gpu_device, S, depth):
    from emqx_amd import workload as W
    fb, fo = W.filters(1)
    batches = [W.topics(1, n=6000 + 777 * r, stream=r) for r in range(S)]
    got = _run(fb, fo, batches, S, depth)
    _check(fb, fo, batches, got)


def test_routed_golden_vectors(gpu_device):
    """the committed O1 vectors: '$' topics vs root wildcards, '#' parents,
    empty levels, literal '+' / '#' topic levels, long topics"""
    from emqx_amd.engine import pack
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "o1_vectors.json")))
    for vec in g:
        fb, fo = pack([f.encode(L1) for f in vec["filters"]])
        topics = [r["topic"].encode(L1) for r in vec["topics"]]
        for S, depth in ((2, 1), (3, 2)):
            batches = [pack(topics[r::S]) for r in range(S)]
            got = _run(fb, fo, batches, S, depth)
            for r in range(S):
                c, oo, ids = got[r]
                rows = vec["topics"][r::S]
                for t, row in enumerate(rows):
                    want = row["match"]
                    have = [vec["filters"][int(i)] for i in ids[oo[t]:oo[t + 1]]]
                    assert have == want, (vec["name"], row["topic"], S, depth)


def test_routed_c2_sample_and_empty_rank(gpu_device):
    """a larger trie (C2: 1M filters), ranks of unequal batch sizes, one rank
    with an empty batch"""
    from emqx_amd import workload as W
    fb, fo = W.filters(2, n=300_000)
    batches = [W.topics(2, n=20000, stream=7), W.topics(2, n=0, stream=8), W.topics(2, n=5000, stream=9)]
    got = _run(fb, fo, batches, 3, 2)
    _check(fb, fo, batches, got)


@pytest.mark.parametrize("self_rccl", [False, True])
def test_route_exchange_one_rank_rccl_equals_o1(gpu_device, self_rccl):
    """the multi-process entry points tm_route_exchange / tm_route_return (one
    rank per process, as bench.py --mode routed runs them) on a one-rank RCCL
    communicator: plan, size all-to-all, transfers, receive scan, the owner's
    walk, the return and the unpermute.  self_rccl: the rank's own buckets go
    through ncclSend / ncclRecv to itself and the size exchanges through
    ncclAllToAll, i.e. the RCCL code the ranks of a multi-GPU node run."""
    import torch
    from emqx_amd import shard
    from emqx_amd import workload as W
    from emqx_amd.engine import check_total
    fb, fo = W.filters(1)
    tb, to = W.topics(1, n=9000, stream=4)
    comm = shard.Comm.init_rank(shard.Comm.unique_id(), 1, 0, gpu_device)
    assert comm.rccl
    if self_rccl:
        comm.set_self_rccl(True)
    e = shard.RoutedEngine(gpu_device, 1, 0, depth=2)
    e.insert_many(fb, fo)
    e.commit()
    dev = torch.device("cuda", gpu_device)
    st = torch.cuda.Stream(device=dev)
    pad = np.zeros(len(tb) + 16, dtype=np.uint8)
    pad[:len(tb)] = tb
    d_b = torch.from_numpy(pad).to(dev)
    d_o = torch.from_numpy(np.ascontiguousarray(to).view(np.int64).copy()).to(dev)
    n = len(to) - 1
    for rep in range(2):
        o = shard.route_exchange(comm, shard.route_in(n, int(to[-1]), d_b, d_o, 2, st))
        assert o.m == n and o.bytes == int(to[-1])
        c = torch.empty(o.m, dtype=torch.int32, device=dev)
        oo = torch.empty(o.m + 1, dtype=torch.int64, device=dev)
        t = torch.zeros(1, dtype=torch.int64, device=dev)
        e.match_batch_device(o.d_bytes, o.d_off, o.m, o.bytes, c, oo, None, 0, t, stream=st)
        st.synchronize()
        cap = int(t.item()) + 1
        ids = torch.empty(cap, dtype=torch.int32, device=dev)
        e.match_batch_device(o.d_bytes, o.d_off, o.m, o.bytes, c, oo, ids, cap, t, stream=st)
        st.synchronize()
        check_total(t, cap)
        r = shard.route_return(comm, c, oo, ids, stream=st)
        st.synchronize()
        got = (shard._dev_array(r.d_counts, r.n, np.uint32, gpu_device),
               shard._dev_array(r.d_offs, r.n + 1, np.uint64, gpu_device),
               shard._dev_array(r.d_ids, r.total, np.uint32, gpu_device))
        _check(fb, fo, [(tb, to)], [got])
    comm.close()
    e.close()


def test_routed_64_shards_one_gpu_equals_o1(gpu_device):
    """MAX_ROUTE_SHARDS = 64 shards (the plan's S + 1 = 65 bucket
    cuts used to be gathered by one 64-lane block, leaving the last cut
    unwritten): every rank's lists equal O1; most shards own few or no topics"""
    from emqx_amd import workload as W
    fb, fo = W.filters(1)
    S = 64
    batches = [W.topics(1, n=(300 if r % 7 else 0) + 11 * r, stream=100 + r) for r in range(S)]
    got = _run(fb, fo, batches, S, 2)
    _check(fb, fo, batches, got)
