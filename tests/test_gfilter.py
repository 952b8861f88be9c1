"""Per-node filters of the big WIDE nodes (option "gfilter", image.h
gf_word), host side: after relayouts and through inserts / deletes between
them, every literal child of a classed node is in the node's filter region
(a filter may only pass too much, never too little) and every reference
carries its node's class (tm_debug_check_filters).  The walk's use of them
is checked on the GPU by test_gpu_parity's gfilter variants (the option
is off by default: at C3 the filter loads cost more than the probes they
save)."""
import ctypes
import random

from emqx_amd import Engine
from emqx_amd import workload as W


def check(eng):
    f = eng.lib.tm_debug_check_filters
    f.restype = ctypes.c_int
    assert f(eng.h) == 0


def test_filters_consistent_through_churn():
    rng = random.Random(5)
    eng = Engine(device=-1)
    eng.set_option("gfilter", 1)
    # big nodes: 'a/<k>' for 300 words, 'b/<k>/x' for 40, 'c/+/<k>' for 20
    base = [b"a/%d" % k for k in range(300)] + [b"b/%d/x" % k for k in range(40)] + \
           [b"c/+/%d" % k for k in range(20)] + [b"d/%d/#" % k for k in range(70)]
    for f in base:
        eng.insert(f)
    eng.commit()
    check(eng)
    live = set(base)
    for rnd in range(6):
        adds = [b"%s/%d" % (rng.choice([b"a", b"b/3", b"c/+", b"d", b"e"]), rng.randrange(2000)) for _ in range(400)]
        for f in adds:
            eng.insert(f)
            live.add(f)
        for f in rng.sample(sorted(live), 150):
            eng.delete(f)
            live.discard(f)
        check(eng)        # between relayouts: new children in old regions
        eng.commit()
        check(eng)
    eng.set_option("relayout", 1)
    eng.commit()
    check(eng)
    eng.close()


def test_filters_on_c1_and_off():
    fb, fo = W.filters(1)
    for on in (1, 0):
        eng = Engine(device=-1)
        eng.set_option("gfilter", on)
        eng.insert_many(fb, fo)
        eng.commit()
        check(eng)
        eng.close()
