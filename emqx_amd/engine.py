"""Python handle on one libtopicmatch engine (one engine per GPU).

Thin wrapper over the C-ABI: numpy arrays for host batches, torch tensors
(or raw device pointers) for HBM-resident batches.  No matching logic lives
here; every match runs in the HIP kernels of emqx_amd/csrc/kernels.hip.
"""
import ctypes

import numpy as np

from . import _lib as L


def pack(strings):
    """Concatenate byte strings -> (bytes ndarray u8, offsets ndarray u64)."""
    bs = [s if isinstance(s, (bytes, bytearray)) else s.encode() for s in strings]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bs) + b"\0" * 8, dtype=np.uint8)
    return buf, off


def check_total(d_total, cap, what="match"):
    """the exact total a two-pass device call wrote (a 1-element device tensor
    whose stream the caller has synchronised) against the capacity of the
    output it sized from the first pass: the device API drops ids past cap and
    reports the exact total, so a total past cap means lists were cut (e.g. a
    first-pass total overwritten by a late fill) -- raise instead of
    returning them"""
    total = int(d_total.item()) if hasattr(d_total, "item") else int(d_total)
    if total > cap:
        raise RuntimeError("%s: %d ids past an output of %d (lists would be cut)" % (what, total, cap))
    return total


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class Engine:
    """One subscription trie + its HBM image on `device` (-1 = host-only:
    insert/delete/lookup work, matching raises TM_EDEVICE)."""

    def __init__(self, device=0, filters_hint=0, batch_topics=0, batch_bytes=0, devices=None):
        """devices: a list of HIP ordinals opens one engine with a replica on
        each (tm_open_devices; host batches are cut across them)"""
        self.lib = L.load()
        cfg = L.TmConfig(device, 0, filters_hint, batch_topics, batch_bytes)
        h = ctypes.c_void_p()
        if devices is not None:
            arr = (ctypes.c_int32 * max(len(devices), 1))(*devices)
            rc = self.lib.tm_open_devices(ctypes.byref(cfg), arr, len(devices), ctypes.byref(h))
            what = "tm_open_devices(%s)" % list(devices)
            device = devices[0] if devices else -1
        else:
            rc = self.lib.tm_open(ctypes.byref(cfg), ctypes.byref(h))
            what = "tm_open(device=%d)" % device
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, what)
        self.h = h
        self.device = device

    @property
    def replicas(self):
        return self.lib.tm_engine_replicas(self.h)

    # -- lifetime ---------------------------------------------------------
    def close(self):
        if self.h:
            self.lib.tm_close(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "%s: %s" % (what, self.lib.tm_last_error(self.h).decode()))
        return rc

    # -- emqx_trie:insert/1, delete/1, lookup/1 ---------------------------
    def insert(self, filt: bytes):
        return self._check(self.lib.tm_insert(self.h, filt, len(filt)), "tm_insert")

    def insert_many(self, buf, off):
        n = len(off) - 1
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        return self._check(self.lib.tm_insert_batch(self.h, _ptr(buf), _ptr(off), n), "tm_insert_batch")

    def insert_many_ids(self, buf, off, ids):
        """tm_insert_batch_ids: filter i under the caller's (global) id ids[i]"""
        n = len(off) - 1
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        return self._check(self.lib.tm_insert_batch_ids(self.h, _ptr(buf), _ptr(off), n, _ptr(ids)),
                           "tm_insert_batch_ids")

    def delete(self, filt: bytes):
        return self._check(self.lib.tm_delete(self.h, filt, len(filt)), "tm_delete")

    def delete_many(self, buf, off):
        n = len(off) - 1
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        return self._check(self.lib.tm_delete_batch(self.h, _ptr(buf), _ptr(off), n), "tm_delete_batch")

    def lookup(self, node_id: bytes):
        """[] or [(edge_count, topic_bytes_or_None)] like emqx_trie:lookup/1"""
        info = L.TmNodeInfo()
        rc = self.lib.tm_lookup(self.h, node_id, len(node_id), ctypes.byref(info))
        if rc == L.TM_ENOENT:
            return []
        self._check(rc, "tm_lookup")
        topic = None if info.filter_id == L.TM_NO_FILTER else self.filter_bytes(info.filter_id)
        return [(info.edge_count, topic)]

    def lease(self):
        """a filter id lease (tm_lease_begin/end), as a context manager: ids
        returned by matches inside it keep naming their filters (a deleted
        filter's id is not reused, its bytes stay gatherable) until it ends"""
        eng = self

        class _Lease:
            def __enter__(self):
                x = ctypes.c_uint64()
                eng._check(eng.lib.tm_lease_begin(eng.h, ctypes.byref(x)), "tm_lease_begin")
                self.x = x.value
                return self

            def __exit__(self, *a):
                eng.lib.tm_lease_end(eng.h, self.x)
        return _Lease()

    def commit(self):
        ep = ctypes.c_uint64()
        self._check(self.lib.tm_commit(self.h, ctypes.byref(ep)), "tm_commit")
        return ep.value

    def filter_bytes(self, fid: int) -> bytes:
        n = ctypes.c_uint32()
        p = self.lib.tm_filter_bytes(self.h, fid, ctypes.byref(n))
        if not p:
            raise KeyError(fid)
        return ctypes.string_at(p, n.value)

    @property
    def filter_count(self):
        return self.lib.tm_filter_count(self.h)

    @property
    def node_count(self):
        return self.lib.tm_node_count(self.h)

    @property
    def image_bytes(self):
        return self.lib.tm_image_bytes(self.h)

    # -- emqx_trie:match/1 over a batch ------------------------------------
    def match_batch(self, buf, off, out_cap=None, counts=None, offs=None, keep=False):
        """Host batch -> (counts u32[n], offsets u64[n+1], filter ids u32[total]).
        counts / offs: caller arrays to fill (e.g. pinned); keep=True returns
        the ids as a view of the library's pinned output buffer, released
        when the array is garbage-collected (no copy)."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) - 1
        counts = np.zeros(max(n, 1), dtype=np.uint32) if counts is None else counts
        offs = np.zeros(n + 1, dtype=np.uint64) if offs is None else offs
        if out_cap is None:   # library-sized output: one walk, no retry (tm_match_batch_owned)
            p, total = ctypes.c_void_p(), ctypes.c_uint64()
            rc = self.lib.tm_match_batch_owned(self.h, _ptr(buf), _ptr(off), n, _ptr(counts), _ptr(offs),
                                               ctypes.byref(p), ctypes.byref(total))
            if rc != L.TM_OK:
                self.lib.tm_free(p)
                self._check(rc, "tm_match_batch_owned")
            k = int(total.value)
            ids = np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_uint32)), shape=(max(k, 1),))
            if keep:
                import weakref
                view = ids[:k]
                weakref.finalize(view, self.lib.tm_free, ctypes.c_void_p(p.value))
                return counts[:n], offs, view
            try:
                return counts[:n], offs, ids[:k].copy()
            finally:
                self.lib.tm_free(p)
        ids = np.zeros(max(out_cap, 1), dtype=np.uint32)
        needed = ctypes.c_uint64()
        rc = self.lib.tm_match_batch(self.h, _ptr(buf), _ptr(off), n, _ptr(counts), _ptr(offs), _ptr(ids),
                                     out_cap, ctypes.byref(needed))
        self._check(rc, "tm_match_batch")
        return counts[:n], offs, ids[: int(needed.value)]

    def filters_bytes(self, ids):
        """bytes of many filter ids, copied under the engine lock (tm_filters_gather)"""
        ids = np.ascontiguousarray(ids, dtype=np.uint32)
        n = len(ids)
        off = np.zeros(n + 1, dtype=np.uint64)
        cap = n * 48 + 64
        while True:
            buf = np.zeros(max(cap, 1), dtype=np.uint8)
            rc = self.lib.tm_filters_gather(self.h, _ptr(ids), n, _ptr(buf), cap, _ptr(off))
            if rc == L.TM_ENOSPC:
                cap = int(off[-1])
                continue
            self._check(rc, "tm_filters_gather")
            b = buf.tobytes()
            return [b[int(off[i]):int(off[i + 1])] for i in range(n)]

    def match(self, topics):
        """list of topics -> list of lists of filter bytes, reference order."""
        buf, off = pack(topics)
        counts, offs, ids = self.match_batch(buf, off)
        uniq, inv = np.unique(ids, return_inverse=True)
        names = self.filters_bytes(uniq)
        out = []
        for t in range(len(topics)):
            a, b = int(offs[t]), int(offs[t]) + int(counts[t])
            out.append([names[int(k)] for k in inv[a:b]])
        return out

    def match_batch_device(self, d_bytes, d_off, n, topic_bytes, d_counts, d_offs, d_ids, out_cap, d_total,
                           stream=None):
        """All arguments are device pointers (ints) or torch tensors; stream-
        ordered, no synchronisation."""
        def p(x):
            if x is None:
                return None
            if hasattr(x, "data_ptr"):
                return ctypes.c_void_p(x.data_ptr())
            return ctypes.c_void_p(int(x))
        st = None
        if stream is not None:
            st = ctypes.c_void_p(L.stream_handle(stream))
        rc = self.lib.tm_match_batch_device(self.h, p(d_bytes), p(d_off), n, topic_bytes, p(d_counts), p(d_offs),
                                            p(d_ids), out_cap, p(d_total), st)
        return self._check(rc, "tm_match_batch_device")

    def match_small_device(self, d_bytes, d_off, n, topic_bytes, d_counts, d_offs, d_ids, out_cap, d_total,
                           stream=None):
        """tm_match_small_device: the lists of a small batch in one launch;
        topic t's list is d_ids[d_offs[t] : d_offs[t] + d_counts[t]] (lists
        in completion order, d_offs has n entries)"""
        def p(x):
            if x is None:
                return None
            if hasattr(x, "data_ptr"):
                return ctypes.c_void_p(x.data_ptr())
            return ctypes.c_void_p(int(x))
        st = None if stream is None else ctypes.c_void_p(L.stream_handle(stream))
        rc = self.lib.tm_match_small_device(self.h, p(d_bytes), p(d_off), n, topic_bytes, p(d_counts), p(d_offs),
                                            p(d_ids), out_cap, p(d_total), st)
        return self._check(rc, "tm_match_small_device")

    # -- emqx_router: the route bag and match_routes/1 ----------------------
    TOPIC_ROUTE = 0xFFFFFFFF    # route source = the publish topic itself

    def route_add(self, topic: bytes, dest: bytes):
        return self._check(self.lib.tm_route_add(self.h, topic, len(topic), dest, len(dest)), "tm_route_add")

    def route_add_many(self, tbuf, toff, dbuf, doff):
        """route i = (topic i of (tbuf, toff), dest i of (dbuf, doff))"""
        n = len(toff) - 1
        tbuf = np.ascontiguousarray(tbuf, dtype=np.uint8)
        toff = np.ascontiguousarray(toff, dtype=np.uint64)
        dbuf = np.ascontiguousarray(dbuf, dtype=np.uint8)
        doff = np.ascontiguousarray(doff, dtype=np.uint64)
        return self._check(self.lib.tm_route_add_batch(self.h, _ptr(tbuf), _ptr(toff), _ptr(dbuf), _ptr(doff), n),
                           "tm_route_add_batch")

    def route_del(self, topic: bytes, dest: bytes):
        return self._check(self.lib.tm_route_del(self.h, topic, len(topic), dest, len(dest)), "tm_route_del")

    def route_del_many(self, tbuf, toff, dbuf, doff):
        """route i = (topic i of (tbuf, toff), dest i of (dbuf, doff)), removed in order"""
        n = len(toff) - 1
        tbuf = np.ascontiguousarray(tbuf, dtype=np.uint8)
        toff = np.ascontiguousarray(toff, dtype=np.uint64)
        dbuf = np.ascontiguousarray(dbuf, dtype=np.uint8)
        doff = np.ascontiguousarray(doff, dtype=np.uint64)
        return self._check(self.lib.tm_route_del_batch(self.h, _ptr(tbuf), _ptr(toff), _ptr(dbuf), _ptr(doff), n),
                           "tm_route_del_batch")

    # the emqx_route table events of the delta feed (route bag only, never
    # the trie: emqx_trie_gpu_feed.erl drives the trie from emqx_trie_node)
    def route_write(self, topic: bytes, dest: bytes):
        """mnesia:write(emqx_route, #route{}) (add_trie_route/1 :231, add_direct_route/1 :223-224)"""
        return self._check(self.lib.tm_route_write(self.h, topic, len(topic), dest, len(dest)), "tm_route_write")

    def route_delete_object(self, topic: bytes, dest: bytes):
        """mnesia:delete_object(emqx_route, #route{}) (del_trie_route/1 :255-258,
        emqx_router_helper:cleanup_routes/1 :156-160): the filter stays in the trie"""
        return self._check(self.lib.tm_route_delete_object(self.h, topic, len(topic), dest, len(dest)),
                           "tm_route_delete_object")

    def route_write_many(self, tbuf, toff, dbuf, doff):
        n = len(toff) - 1
        tbuf = np.ascontiguousarray(tbuf, dtype=np.uint8)
        toff = np.ascontiguousarray(toff, dtype=np.uint64)
        dbuf = np.ascontiguousarray(dbuf, dtype=np.uint8)
        doff = np.ascontiguousarray(doff, dtype=np.uint64)
        return self._check(self.lib.tm_route_write_batch(self.h, _ptr(tbuf), _ptr(toff), _ptr(dbuf), _ptr(doff), n),
                           "tm_route_write_batch")

    def get_routes(self, topic: bytes):
        """dest ids of topic's routes, insertion order (get_routes/1)"""
        n = ctypes.c_uint32()
        cap = 16
        while True:
            out = np.zeros(cap, dtype=np.uint32)
            rc = self.lib.tm_get_routes(self.h, topic, len(topic), out.ctypes.data, cap, ctypes.byref(n))
            if rc == L.TM_ENOSPC:
                cap = n.value
                continue
            self._check(rc, "tm_get_routes")
            return [int(x) for x in out[: n.value]]

    @property
    def route_count(self):
        return self.lib.tm_route_count(self.h)

    def dest_bytes(self, dest_id: int) -> bytes:
        n = ctypes.c_uint32()
        p = self.lib.tm_dest_bytes(self.h, dest_id, ctypes.byref(n))
        if not p:
            raise KeyError(dest_id)
        return ctypes.string_at(p, n.value)

    def match_routes_batch(self, buf, off, out_cap=None):
        """Host batch -> (counts u32[n], offsets u64[n+1], src u32[total],
        dest u32[total]): emqx_router:match_routes/1 per topic, src =
        TOPIC_ROUTE for the literal topic's routes, else the filter id."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) - 1
        counts = np.zeros(max(n, 1), dtype=np.uint32)
        offs = np.zeros(n + 1, dtype=np.uint64)
        cap = 1 << 16 if out_cap is None else out_cap
        while True:
            src = np.zeros(max(cap, 1), dtype=np.uint32)
            dst = np.zeros(max(cap, 1), dtype=np.uint32)
            needed = ctypes.c_uint64()
            rc = self.lib.tm_match_routes_batch(self.h, _ptr(buf), _ptr(off), n, _ptr(counts), _ptr(offs), _ptr(src),
                                                _ptr(dst), cap, ctypes.byref(needed))
            if rc == L.TM_ENOSPC and out_cap is None:
                cap = int(needed.value)
                continue
            self._check(rc, "tm_match_routes_batch")
            k = int(needed.value)
            return counts[:n], offs, src[:k], dst[:k]

    def match_routes_batch_device(self, d_bytes, d_off, n, topic_bytes, d_counts, d_offs, d_src, d_dest, out_cap,
                                  d_total, stream=None):
        def p(x):
            if x is None:
                return None
            return ctypes.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))
        st = None
        if stream is not None:
            st = ctypes.c_void_p(L.stream_handle(stream))
        rc = self.lib.tm_match_routes_batch_device(self.h, p(d_bytes), p(d_off), n, topic_bytes, p(d_counts),
                                                   p(d_offs), p(d_src), p(d_dest), out_cap, p(d_total), st)
        return self._check(rc, "tm_match_routes_batch_device")

    # -- emqx_broker:aggre/1 (aggre.hip) --------------------------------------
    TARGET_NODE, TARGET_GROUP = 0, 1

    def debug_check_routes(self):
        """host-side consistency check of the in-place route image (diagnostic,
        tm_debug_check_routes): raises TopicMatchError naming the first defect"""
        return self._check(self.lib.tm_debug_check_routes(self.h), "tm_debug_check_routes")

    def dest_target(self, dest: bytes, kind: int, key: bytes) -> int:
        """declare dest's aggre target: a node atom (TARGET_NODE, key = its
        text) or a $share group (TARGET_GROUP, key = the group binary)"""
        t = ctypes.c_uint32()
        self._check(self.lib.tm_dest_target(self.h, dest, len(dest), kind, key, len(key), ctypes.byref(t)),
                    "tm_dest_target")
        return t.value

    def target_bytes(self, target_id: int):
        """target id -> (kind, key bytes)"""
        kind, n = ctypes.c_uint32(), ctypes.c_uint32()
        p = self.lib.tm_target_bytes(self.h, target_id, ctypes.byref(kind), ctypes.byref(n))
        if not p:
            raise KeyError(target_id)
        return kind.value, ctypes.string_at(p, n.value)

    def match_deliveries_batch(self, buf, off, out_cap=None):
        """Host batch -> (counts u32[n], offsets u64[n+1], to u32[total],
        target u32[total]): aggre(emqx_router:match_routes(T)) per topic; to =
        TOPIC_ROUTE for the literal topic, else the filter id."""
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        n = len(off) - 1
        counts = np.zeros(max(n, 1), dtype=np.uint32)
        offs = np.zeros(n + 1, dtype=np.uint64)
        cap = 1 << 16 if out_cap is None else out_cap
        while True:
            to = np.zeros(max(cap, 1), dtype=np.uint32)
            tg = np.zeros(max(cap, 1), dtype=np.uint32)
            needed = ctypes.c_uint64()
            rc = self.lib.tm_match_deliveries_batch(self.h, _ptr(buf), _ptr(off), n, _ptr(counts), _ptr(offs),
                                                    _ptr(to), _ptr(tg), cap, ctypes.byref(needed))
            if rc == L.TM_ENOSPC and out_cap is None:
                cap = int(needed.value)
                continue
            self._check(rc, "tm_match_deliveries_batch")
            k = int(needed.value)
            return counts[:n], offs, to[:k], tg[:k]

    def match_deliveries_batch_device(self, d_bytes, d_off, n, topic_bytes, d_counts, d_offs, d_to, d_target,
                                      out_cap, d_total, stream=None):
        def p(x):
            if x is None:
                return None
            return ctypes.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))
        st = None
        if stream is not None:
            st = ctypes.c_void_p(L.stream_handle(stream))
        rc = self.lib.tm_match_deliveries_batch_device(self.h, p(d_bytes), p(d_off), n, topic_bytes, p(d_counts),
                                                       p(d_offs), p(d_to), p(d_target), out_cap, p(d_total), st)
        return self._check(rc, "tm_match_deliveries_batch_device")

    # walk variants (A/B knobs of tm_walk_queue): one global dequeue head, or
    # per-XCD heads over contiguous ranges of the batch
    WALKS = {"queue": 0, "queue_xcd": 1}

    def set_option(self, name: str, value: int):
        self._check(self.lib.tm_set_option(self.h, name.encode(), int(value)), "tm_set_option(%s)" % name)

    def set_walk(self, walk: str):
        self.set_option("xcdq", self.WALKS[walk])

    # -- instrumentation ----------------------------------------------------
    def set_stats(self, on=True):
        self._check(self.lib.tm_set_stats(self.h, 1 if on else 0), "tm_set_stats")

    def last_stats(self):
        s = L.TmBatchStats()
        self._check(self.lib.tm_last_stats(self.h, ctypes.byref(s)), "tm_last_stats")
        return {k: getattr(s, k) for k, _ in s._fields_}

    def set_timing(self, on=True):
        self._check(self.lib.tm_set_timing(self.h, 1 if on else 0), "tm_set_timing")

    def last_kernel_times(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        k = self.lib.tm_last_kernel_times(self.h, names, ms, 16)
        if k < 0:
            self._check(k, "tm_last_kernel_times")
        return {names[i].decode(): ms[i] for i in range(k)}
