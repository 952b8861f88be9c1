"""libtopicmatch host logic without a GPU: the C-ABI loads and exports every
declared symbol, the trie bookkeeping (insert/delete/lookup, emqx_trie.erl
:62-117, :149-163) matches the reference's KATs and the pytrie transcription,
and the match path refuses to run host-only (no CPU fallback)."""
import os
import random
import re

import pytest

from emqx_amd import Engine, _lib
from emqx_amd.engine import pack
from emqx_amd.emqx_router import Router
from oracle import pytrie

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L1 = "latin-1"


def b(x):
    return x.encode(L1)


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "topicmatch.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(tm_[a-z_]+)\s*\(", txt)))


def test_abi_exports_every_header_symbol():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 20
    bound = {name for name, _, _ in _lib.SIGNATURES}
    for s in syms:
        assert hasattr(lib, s), s
        assert s in bound, "no ctypes signature for %s" % s
    assert "gfx950" in lib.tm_build_info().decode()


def test_library_code_objects_are_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    for other in (b"gfx942", b"gfx90a", b"sm_"):
        assert b"amdgcn-amd-amdhsa--" + other not in blob


def test_strerror_codes():
    lib = _lib.load()
    for code in range(-6, 1):
        assert lib.tm_strerror(code).decode() != "unknown status"


def kat_engine():
    return Engine(device=-1)


def test_kat_trie_bookkeeping(golden):
    for kat in golden["kat_trie"]:
        e = kat_engine()
        for op, arg in kat["ops"]:
            getattr(e, op)(b(arg))
        for kind, arg, exp in kat["checks"]:
            if kind == "lookup":
                got = [[ec, None if t is None else t.decode(L1)] for ec, t in e.lookup(b(arg))]
                assert got == exp, (kat["name"], arg, got)
        e.close()


def test_match_refuses_host_only():
    e = kat_engine()
    e.insert(b"a/#")
    with pytest.raises(_lib.TopicMatchError) as ei:
        e.match([b"a/b"])
    assert ei.value.code == _lib.TM_EDEVICE


def test_filter_ids_and_bytes():
    e = kat_engine()
    for f in [b"a/+", b"a/#", b"#", b"", b"a//b"]:
        e.insert(f)
    assert e.filter_count == 5
    e.insert(b"a/+")                     # idempotent
    assert e.filter_count == 5
    for f in [b"a/+", b"a/#", b"#", b"", b"a//b"]:
        (ec, topic), = e.lookup(f)
        assert topic == f
    e.delete(b"a/#")
    assert e.lookup(b"a/#") == []
    assert e.filter_count == 4
    e.delete(b"nope/#")                  # unknown: no-op
    assert e.filter_count == 4


def _prefixes(f):
    parts = f.split(b"/")
    return [b"/".join(parts[:k]) for k in range(1, len(parts) + 1)]


def test_bookkeeping_vs_pytrie_random():
    rng = random.Random(2024)
    for _ in range(40):
        e, py = kat_engine(), pytrie.Trie()
        pool = []
        for _ in range(rng.randint(5, 80)):
            k = rng.randint(1, 6)
            pool.append(b"/".join(rng.choice([b"a", b"b", b"", b"+", b"#", b"$x", b"c"]) for _ in range(k)))
        live = set()
        for _ in range(200):
            f = rng.choice(pool)
            if rng.random() < 0.6:
                e.insert(f)
                py.insert(f)
                live.add(f)
            else:
                e.delete(f)
                py.delete(f)
                live.discard(f)
        for f in pool:
            for nid in _prefixes(f):
                assert e.lookup(nid) == py.lookup(nid), nid
        e.close()


def test_router_kat_host_side(golden):
    """route-table bookkeeping of emqx_router (add/del with trie deltas);
    the match itself needs the GPU and is covered by the gpu suite"""
    for kat in golden["kat_router"]:
        r = Router(kat_engine(), node="node")
        for topic, dest in kat["add"]:
            r.add_route(b(topic), dest)
        assert sorted(t.decode() for t in r.topics()) == sorted({t for t, _ in kat["add"]})
        for topic, _ in kat["add"]:
            if "+" in topic or "#" in topic:
                assert r.engine.lookup(b(topic))[0][1] == b(topic)
        if "then_del" in kat:
            for topic, dest in kat["then_del"]:
                r.del_route(b(topic), dest)
            node, exp = kat["lookup_after"]
            assert r.engine.lookup(b(node)) == exp


@pytest.mark.parametrize("hot,hot_edges,order", [(0, 0, 0), (1, 3, 1), (3, 2, 2), (3, 3, 3), (4, 5, 1), (4, 0, 5),
                                                 (0, 0, 7)])
def test_relayout_preserves_bookkeeping(hot, hot_edges, order):
    """DFS-preorder relayout on every commit (layout=2), with depths <= hot
    laid out level by level first ('+' child first / '#' nodes last / heat
    order per `order`), keeps emqx_trie's bookkeeping (edge_count, topic)
    and the filter ids intact"""
    rng = random.Random(31 + hot + 7 * hot_edges + 101 * order)
    for _ in range(25):
        e, py = kat_engine(), pytrie.Trie()
        e.set_option("layout", 2)
        e.set_option("hot_levels", hot)
        e.set_option("hot_edges", hot_edges)
        e.set_option("order", order)
        e.set_option("edge_load", 2 + (order % 3) * 3)
        pool = [b"/".join(rng.choice([b"a", b"b", b"", b"+", b"#", b"$x", b"c", b"d", b"e"])
                          for _ in range(rng.randint(1, 6))) for _ in range(rng.randint(5, 120))]
        for step in range(300):
            f = rng.choice(pool)
            if rng.random() < 0.6:
                e.insert(f)
                py.insert(f)
            else:
                e.delete(f)
                py.delete(f)
            if step % 37 == 0:
                e.commit()
        e.commit()
        for f in pool:
            for nid in _prefixes(f):
                assert e.lookup(nid) == py.lookup(nid), nid
        e.close()


def test_filters_and_dests_gather():
    """tm_filters_gather / tm_dests_gather copy under the engine lock; ENOSPC
    reports the bytes needed; unknown ids are refused"""
    e = Engine(device=-1)
    fs = [b"a/+", b"", b"b/#", b"+/+/c" * 20]
    for f in fs:
        e.insert(f)                     # filter ids 0..3 in insertion order
    assert e.filters_bytes([0, 1, 2, 3]) == fs
    assert e.filters_bytes([3, 3, 0]) == [fs[3], fs[3], fs[0]]
    assert e.filters_bytes([]) == []
    import ctypes
    off = (ctypes.c_uint64 * 3)()
    buf = (ctypes.c_uint8 * 4)()
    idarr = (ctypes.c_uint32 * 2)(3, 0)
    assert e.lib.tm_filters_gather(e.h, idarr, 2, buf, 4, off) == _lib.TM_ENOSPC
    assert off[2] == len(fs[3]) + len(fs[0])
    bad = (ctypes.c_uint32 * 1)(99)
    assert e.lib.tm_filters_gather(e.h, bad, 1, buf, 4, off) == _lib.TM_EINVAL
    e.route_add(b"a/+", b"node1")
    e.route_add(b"x", b"node2")
    d = (ctypes.c_uint32 * 2)(1, 0)
    big = (ctypes.c_uint8 * 64)()
    assert e.lib.tm_dests_gather(e.h, d, 2, big, 64, off) == _lib.TM_OK
    assert bytes(big[:off[2]]) == b"node2node1"
    e.close()


def test_open_devices_host_only_and_bad_ordinals():
    import ctypes
    from emqx_amd import _lib as L
    e = Engine(devices=[])           # no replica: host-only
    assert e.replicas == 0
    e.insert(b"a/+")
    with pytest.raises(L.TopicMatchError) as ex:
        e.match_batch(*pack([b"a/b"]))
    assert ex.value.code == L.TM_EDEVICE
    e.close()
    lib = L.load()
    h = ctypes.c_void_p()
    cfg = L.TmConfig(-1, 0, 0, 0, 0)
    arr = (ctypes.c_int32 * 1)(-5)
    assert lib.tm_open_devices(ctypes.byref(cfg), arr, 1, ctypes.byref(h)) in (L.TM_EDEVICE, L.TM_EINVAL)
