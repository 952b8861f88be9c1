"""Publish micro-batcher (include/topicmatch.h tm_batcher_*).

Many publisher threads submit single topics; the native worker thread seals
device batches (by size or deadline) and calls back once per topic with its
ordered match list (emqx_trie:match/1 filter ids), its match_routes/1
routes, or (deliveries=True) aggre(match_routes/1): To ids + target ids.  This is the NIF's path: the callback there builds
the Erlang list and enif_send()s it to the waiting process."""
import ctypes
import itertools

from . import _lib as L


class Batcher:
    def __init__(self, engine, max_topics=65536, deadline_us=200, max_bytes=0, routes=False, deliveries=False,
                 lanes_per_replica=0, callback_threads=0):
        self.engine = engine
        self.lib = engine.lib
        flags = (L.TM_BATCHER_ROUTES if routes else 0) | (L.TM_BATCHER_DELIVERIES if deliveries else 0)
        cfg = L.TmBatcherConfig(max_topics, deadline_us, max_bytes, flags, lanes_per_replica, callback_threads)
        h = ctypes.c_void_p()
        rc = self.lib.tm_batcher_open(engine.h, ctypes.byref(cfg), ctypes.byref(h))
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_batcher_open")
        self.h = h
        self.routes = routes
        self._cbs = {}
        self._keys = itertools.count(1)
        self._done = L.DONE_FN(self._on_done)     # one trampoline, kept alive with the batcher

    def _on_done(self, ctx, ticket, status, ids, dests, n):
        cb = self._cbs.pop(ctx)
        if status != L.TM_OK:
            cb(status, None, None)
            return
        a = [ids[i] for i in range(n)]
        d = [dests[i] for i in range(n)] if dests else None
        cb(status, a, d)

    def submit(self, topic: bytes, callback):
        """callback(status, ids, dests) runs on the worker thread"""
        t = ctypes.c_uint64()
        key = next(self._keys)              # the callback may fire before submit returns
        self._cbs[key] = callback
        rc = self.lib.tm_batcher_submit(self.h, topic, len(topic), self._done, key, ctypes.byref(t))
        if rc != L.TM_OK:
            del self._cbs[key]
            raise L.TopicMatchError(rc, "tm_batcher_submit")
        return t.value

    def flush(self):
        rc = self.lib.tm_batcher_flush(self.h)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_batcher_flush")

    def stats(self, reset_max=False):
        """tm_batcher_get_stats2: every counter; the max_* fields cover the
        batches since the open or the last read with reset_max=True"""
        s = L.TmBatcherStats()
        rc = self.lib.tm_batcher_get_stats2(self.h, ctypes.byref(s), ctypes.sizeof(s),
                                            L.TM_BATCHER_STATS_RESET_MAX if reset_max else 0)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_batcher_get_stats2")
        return {k: getattr(s, k) for k, _ in s._fields_}

    def close(self):
        if self.h:
            self.lib.tm_batcher_close(self.h)
            self.h = None
