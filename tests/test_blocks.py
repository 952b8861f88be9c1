"""Per-node child blocks (option "blocks", image.h BlockSlot): the host
mirror's WIDE nodes keep their literal children in blocks of their own.
Host-only here (the -m gpu parity tests run every walk over them): the blocks
stay consistent (tm_debug_check_blocks) through inserts that grow blocks,
deletes that shift and free them, compaction and relayouts in both
directions, and emqx_trie:lookup/1 stays equal to O1 throughout."""
import ctypes
import random

import pytest

from emqx_amd import Engine
from emqx_amd import workload as W
from emqx_amd.engine import pack
from oracle import O1


def check(eng):
    lib = eng.lib
    lib.tm_debug_check_blocks.restype = ctypes.c_int
    rc = lib.tm_debug_check_blocks(eng.h)
    assert rc == 0, eng.lib.tm_last_error(eng.h).decode()


def prefixes(f):
    ws = f.split(b"/")
    return [b"/".join(ws[:i]) for i in range(1, len(ws) + 1)]


def same_lookups(eng, o1, filters):
    for f in filters:
        for p in prefixes(f):
            assert eng.lookup(p) == o1.lookup(p), p


@pytest.mark.parametrize("blocks", [1, 0])
def test_blocks_consistent_under_churn(blocks):
    rng = random.Random(7)
    words = [b"w%d" % i for i in range(40)] + [b"+"]
    pool = set()
    while len(pool) < 3000:
        n = rng.randint(1, 4)
        f = b"/".join(rng.choice(words) for _ in range(n))
        if rng.random() < 0.1:
            f += b"/#"
        pool.add(f)
    pool = sorted(pool)
    eng = Engine(device=-1)
    eng.set_option("blocks", blocks)
    o1 = O1()
    live = set()
    for rnd in range(6):
        ins = rng.sample(pool, 700)
        for f in ins:
            eng.insert(f)
            o1.insert(f)
            live.add(f)
        check(eng)
        dels = rng.sample(sorted(live), min(len(live), 400))
        for f in dels:
            eng.delete(f)
            o1.delete(f)
            live.discard(f)
        check(eng)
        if rnd % 2:
            eng.set_option("relayout", 1)
        eng.commit()
        check(eng)
        same_lookups(eng, o1, rng.sample(pool, 300))
    eng.close()
    o1.close()


def test_blocks_option_converts_both_ways():
    fb, fo = W.filters(1)
    filters = [bytes(x) for x in W.unpack(fb, fo)]
    eng = Engine(device=-1)
    eng.set_option("blocks", 0)
    eng.insert_many(fb, fo)
    eng.commit()
    o1 = O1()
    o1.insert_many(fb, fo)
    for b in (1, 0, 1):
        eng.set_option("blocks", b)
        eng.commit()                          # the relayout converts the representation
        check(eng)
        same_lookups(eng, o1, filters[:500])
        for f in filters[:2000:3]:            # deltas in the new representation
            eng.delete(f)
            o1.delete(f)
        for f in filters[:2000:3]:
            eng.insert(f)
            o1.insert(f)
        check(eng)
        same_lookups(eng, o1, filters[:500])
    eng.close()
    o1.close()


def test_blocks_grow_and_compact():
    """a node with thousands of children: its block doubles again and again
    (each move leaves garbage), then mass deletes; commits compact the pool"""
    eng = Engine(device=-1)
    eng.set_option("blocks", 1)               # an empty trie: blocks from the first insert
    eng.set_option("layout", 0)               # no relayout: growth and compaction only
    eng.set_option("block_gc", 1024)
    o1 = O1()
    fs = [b"hub/c%d/+" % i for i in range(20000)] + [b"hub2/c%d/#" % i for i in range(3000)]
    b, o = pack(fs)
    eng.insert_many(b, o)
    o1.insert_many(b, o)
    check(eng)
    before = eng.image_bytes
    for f in fs[20000:]:                      # hub2's block becomes garbage
        eng.delete(f)
        o1.delete(f)
    for f in fs[:20000:2]:
        eng.delete(f)
        o1.delete(f)
    eng.commit()                              # garbage past half the pool: compacted
    check(eng)
    assert eng.image_bytes < before
    same_lookups(eng, o1, fs[:200])
    eng.close()
    o1.close()
