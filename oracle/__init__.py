"""TEST INFRASTRUCTURE ONLY — the CPU oracle of the topic-routing hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker (never the thing measured on the
GPU, never a fallback of the product path).

    O1      faithful C restatement of emqx_trie (oracle/o1_trie.c)
    O3      the same algorithm over interned word ids and dense node ids
            (oracle/o3_interned.c): the "optimized C++ variant" leg of the
            CPU baseline, checked against O1
    o2_*    brute-force emqx_topic:match/2 scans (same file)
    pytrie  independent pure-Python transcription (oracle/pytrie.py)

Parity pinning: the reference's known-answer tests are transcribed as data in
tests/golden/ (see tests/golden/make_golden.py); O1 and pytrie both reproduce
every vector, and agree with each other on randomized cases.  The Erlang
runtime is absent here, so the reference itself is not executed.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("oracle/liboracle.so not built: run `make`")
    lib = ctypes.CDLL(LIB_PATH)
    V, I, U32, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
    sig = {
        "o1_new": (V, [U64]),
        "o1_free": (None, [V]),
        "o1_insert": (None, [V, ctypes.c_char_p, U32]),
        "o1_insert_batch": (None, [V, V, V, U32]),
        "o1_delete": (I, [V, ctypes.c_char_p, U32]),
        "o1_lookup": (I, [V, ctypes.c_char_p, U32, ctypes.POINTER(U32), ctypes.POINTER(I)]),
        "o1_cursor_new": (V, [V]),
        "o1_cursor_free": (None, [V]),
        "o1_match": (U32, [V, ctypes.c_char_p, U32, ctypes.POINTER(U64)]),
        "o1_cursor_result": (V, [V, U32, ctypes.POINTER(U32)]),
        "o1_match_batch": (ctypes.c_double, [V, V, V, U32, I, V, V, ctypes.POINTER(U64), ctypes.POINTER(U64)]),
        "o1_match_ids": (None, [V, V, V, U32, I, V, V, V]),
        "o1_node_count": (U64, [V]),
        "o1_edge_count": (U64, [V]),
        "o2_topic_match": (I, [ctypes.c_char_p, U32, ctypes.c_char_p, U32]),
        "o3_new": (V, [U64]),
        "o3_free": (None, [V]),
        "o3_insert_batch": (None, [V, V, V, U32]),
        "o3_match_batch": (ctypes.c_double, [V, V, V, U32, I, V, V, V, ctypes.POINTER(U64)]),
        "o2_match": (U32, [V, V, U32, ctypes.c_char_p, U32, V, U32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


class O1:
    """emqx_trie restated over string-path node ids and ETS-like tables."""

    def __init__(self, hint=0):
        self.lib = load()
        self.h = self.lib.o1_new(hint)
        self.cur = self.lib.o1_cursor_new(self.h)

    def close(self):
        if self.h:
            self.lib.o1_cursor_free(self.cur)
            self.lib.o1_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def insert(self, t: bytes):
        self.lib.o1_insert(self.h, t, len(t))

    def insert_many(self, buf, off):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        self.lib.o1_insert_batch(self.h, _p(buf), _p(off), len(off) - 1)

    def delete(self, t: bytes):
        rc = self.lib.o1_delete(self.h, t, len(t))
        if rc != 0:
            raise RuntimeError("mnesia:abort node_not_found")

    def lookup(self, node_id: bytes):
        ec, ht = ctypes.c_uint32(), ctypes.c_int()
        if not self.lib.o1_lookup(self.h, node_id, len(node_id), ctypes.byref(ec), ctypes.byref(ht)):
            return []
        return [(ec.value, node_id if ht.value else None)]

    def match(self, topic: bytes, with_edges=False):
        e = ctypes.c_uint64()
        m = self.lib.o1_match(self.cur, topic, len(topic), ctypes.byref(e))
        out = []
        n = ctypes.c_uint32()
        for i in range(m):
            p = self.lib.o1_cursor_result(self.cur, i, ctypes.byref(n))
            out.append(ctypes.string_at(p, n.value))
        return (out, e.value) if with_edges else out

    def match_batch(self, buf, off, threads=1, per_topic=False):
        """-> (seconds, total_matches, total_edge_reads[, counts, edge_reads])"""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) - 1
        counts = np.zeros(max(n, 1), dtype=np.uint32) if per_topic else None
        edges = np.zeros(max(n, 1), dtype=np.uint64) if per_topic else None
        tm, te = ctypes.c_uint64(), ctypes.c_uint64()
        secs = self.lib.o1_match_batch(self.h, _p(buf), _p(off), n, threads,
                                       _p(counts) if per_topic else None, _p(edges) if per_topic else None,
                                       ctypes.byref(tm), ctypes.byref(te))
        if per_topic:
            return secs, tm.value, te.value, counts[:n], edges[:n]
        return secs, tm.value, te.value

    def match_ids(self, buf, off, threads=1):
        """CSR (counts u32[n], offsets u64[n+1], ids u32[total]) of insertion
        sequence numbers in reference order — comparable 1:1 with the device
        engine's filter ids when both saw the same inserts and no deletes."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) - 1
        counts = np.zeros(max(n, 1), dtype=np.uint32)
        self.lib.o1_match_ids(self.h, _p(buf), _p(off), n, threads, _p(counts), None, None)
        offs = np.zeros(n + 1, dtype=np.uint64)
        offs[1:] = np.cumsum(counts[:n], dtype=np.uint64)
        ids = np.zeros(max(int(offs[-1]), 1), dtype=np.uint32)
        self.lib.o1_match_ids(self.h, _p(buf), _p(off), n, threads, None, _p(offs), _p(ids))
        return counts[:n], offs, ids[: int(offs[-1])]

    @property
    def node_count(self):
        return self.lib.o1_node_count(self.h)


def o2_topic_match(name: bytes, filt: bytes) -> bool:
    return load().o2_topic_match(name, len(name), filt, len(filt)) == 1


def o2_match(filters, topic: bytes):
    """brute force over a list of filters -> set of matching filters"""
    return {f for f in filters if o2_topic_match(topic, f)}


class O3:
    """emqx_trie:match/1 over interned ids (oracle/o3_interned.c): the
    optimized CPU baseline leg; insert-only."""

    def __init__(self, hint=0):
        self.lib = load()
        self.h = self.lib.o3_new(hint)

    def close(self):
        if self.h:
            self.lib.o3_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def insert_many(self, buf, off):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        self.lib.o3_insert_batch(self.h, _p(buf), _p(off), len(off) - 1)

    def match_batch(self, buf, off, threads=1):
        """-> (seconds, total_matches)"""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        tm = ctypes.c_uint64()
        secs = self.lib.o3_match_batch(self.h, _p(buf), _p(off), len(off) - 1, threads, None, None, None,
                                       ctypes.byref(tm))
        return secs, tm.value

    def match_ids(self, buf, off, threads=1):
        """CSR of filter indices (first-insertion order) in reference order"""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) - 1
        counts = np.zeros(max(n, 1), dtype=np.uint32)
        self.lib.o3_match_batch(self.h, _p(buf), _p(off), n, threads, _p(counts), None, None, None)
        offs = np.zeros(n + 1, dtype=np.uint64)
        offs[1:] = np.cumsum(counts[:n], dtype=np.uint64)
        ids = np.zeros(max(int(offs[-1]), 1), dtype=np.uint32)
        self.lib.o3_match_batch(self.h, _p(buf), _p(off), n, threads, None, _p(offs), _p(ids), None)
        return counts[:n], offs, ids[: int(offs[-1])]
