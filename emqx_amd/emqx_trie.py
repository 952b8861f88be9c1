"""emqx_trie — the reference module's API (src/emqx_trie.erl) over the
MI355X engine: same function names, arities and return shapes.

    mnesia(boot | copy)   open the engine (the tables' analogue)
    insert(Topic)         src/emqx_trie.erl:62-73
    match(Topic)          src/emqx_trie.erl:77-79   (HIP kernels on the GPU)
    lookup(NodeId)        src/emqx_trie.erl:83-84   -> [TrieNode] | []
    delete(Topic)         src/emqx_trie.erl:88-96

`TrieNode` mirrors #trie_node{node_id, edge_count, topic, flags}
(include/emqx.hrl:100-105).  A module-level default engine plays the role of
the node-local ram_copies tables; tests and multi-GPU hosts pass `engine=`.
"""
from collections import namedtuple

from .engine import Engine

TrieNode = namedtuple("TrieNode", "node_id edge_count topic flags")

_default = None


def mnesia(mode="boot", device=0, **kw):
    """mnesia(boot) — src/emqx_trie.erl:38-48: create the trie 'tables' (the
    engine with its HBM image).  mnesia(copy) — :50-54: the image is rebuilt
    from the filter registry, so copy == boot here."""
    global _default
    if mode not in ("boot", "copy"):
        raise ValueError(mode)
    if _default is None:
        _default = Engine(device=device, **kw)
    return "ok"


def engine():
    if _default is None:
        mnesia("boot")
    return _default


def _e(engine_):
    return engine_ if engine_ is not None else engine()


def insert(topic: bytes, engine=None):
    _e(engine).insert(topic)
    return "ok"


def delete(topic: bytes, engine=None):
    _e(engine).delete(topic)
    return "ok"


def lookup(node_id: bytes, engine=None):
    r = _e(engine).lookup(node_id)
    return [TrieNode(node_id, ec, topic, None) for ec, topic in r]


def match(topic: bytes, engine=None):
    """-> [filter binaries] in exactly emqx_trie:match/1's order"""
    return _e(engine).match([topic])[0]


def match_many(topics, engine=None):
    """Batched emqx_trie:match/1 (the micro-batcher's entry)."""
    return _e(engine).match(list(topics))
