"""Topic routing by first words (emqx_amd/shard.py routed_partition): the
shard that owns a topic holds every filter that can match it, so its O1
(the restatement of emqx_trie:match/1) returns the full node's list, in the
same order.  CPU only: the design check of a scaling sharded mode."""
import json
import os

import pytest

from emqx_amd import shard
from emqx_amd import workload as W
from oracle import O1

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L1 = "latin-1"


def _check(filters, topics, S, depth):
    full = O1()
    for f in filters:
        full.insert(f)
    per, owner, stats = shard.routed_partition(filters, topics, S, depth)
    shards = []
    for fl in per:
        o = O1()
        for f in fl:
            o.insert(f)
        shards.append(o)
    for t, s in zip(topics, owner):
        assert shards[s].match(t) == full.match(t), (t, s)
    return stats


@pytest.mark.parametrize("S,depth", [(2, 1), (4, 2), (8, 2), (8, 3)])
def test_routed_owner_shard_equals_full_trie_c1(S, depth):
    fb, fo = W.filters(1)
    tb, to = W.topics(1, n=4000)
    filters = [bytes(x) for x in W.unpack(fb, fo)]
    topics = [bytes(x) for x in W.unpack(tb, to)]
    stats = _check(filters, topics, S, depth)
    assert stats["replication"] < S   # literal-led filters live on one shard


def test_routed_owner_shard_equals_full_trie_golden():
    """the committed O1 vectors: '$' topics vs root wildcards, '#' parents,
    empty levels, literal '+' / '#' topic levels, long topics"""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "o1_vectors.json")))
    for vec in g:
        filters = [f.encode(L1) for f in vec["filters"]]
        topics = [r["topic"].encode(L1) for r in vec["topics"]]
        for S, depth in ((3, 1), (5, 2)):
            _check(filters, topics, S, depth)
