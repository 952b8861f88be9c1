"""Sharded mode of the topic-routing engine.

The exchange runs natively over RCCL (emqx_amd/csrc/exchange.cpp):
`Comm.init_rank` + `exchange_native` for one rank per process (the bench and
a broker node with one OS process per GPU), `ShardSet` for all shards of one
process (the C-ABI `tm_comm_init_all` / `tm_shard_exchange_group`; shards
that share a GPU exchange by device copies).  `exchange` below is the
torch.distributed form kept for the gloo CPU tests.

When the filter set is partitioned over S GPUs (one process per GPU), every
GPU holds the sub-trie of its shard (`tm_shard_of`: a hash of the filter's
prefix through its second literal level, so Zipf-heavy root words and
wildcard-led subtrees such as "+/+/..." spread over all shards).  A publish batch is broadcast to all ranks; each rank walks the
WHOLE batch against its sub-trie (match(T, F) = U_s match(T, F_s)) with order
keys (`tm_match_batch_device_keys`), then the ranks exchange per-topic lists
so that rank r ends up owning the complete, ordered match lists of topic slice
r:

    counts  all_to_all_single (slice d of my counts -> rank d)
    sizes   all_to_all_single (how many ids I send to each rank)
    ids     all_to_all_single, uneven splits (RCCL over xGMI on the GPUs)
    keys    all_to_all_single, uneven splits
    merge   tm_shard_merge on the GPU: S key-ordered lists per topic ->
            one list in emqx_trie:match/1 order, global ids local*S + s

An all-to-all moves each id once, to the rank that owns its topic; an
all-gather would move every id to every rank (S x the bytes) only for each
rank to keep 1/S of them.  Ids are global: gid = local_id * S + shard.
"""
import ctypes

import numpy as np

from . import _lib as L
from .engine import Engine, check_total


def shard_of(filt: bytes, n_shards: int) -> int:
    return L.load().tm_shard_of(filt, len(filt), n_shards)


def shard_of_batch(buf, off, n_shards: int):
    """u32[n]: the shard of every filter of a packed batch"""
    n = len(off) - 1
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    out = np.zeros(max(n, 1), dtype=np.uint32)
    rc = L.load().tm_shard_of_batch(buf.ctypes.data, off.ctypes.data, n, n_shards, out.ctypes.data)
    if rc != L.TM_OK:
        raise L.TopicMatchError(rc, "tm_shard_of_batch")
    return out[:n]


def gid_to_index(owner, n_shards: int):
    """For a DISTINCT filter list inserted shard by shard in list order (local
    id = rank among the shard's filters): int64 array gid -> list index, with
    gid = local * n_shards + shard."""
    owner = np.asarray(owner, dtype=np.int64)
    local = np.zeros(len(owner), dtype=np.int64)
    for s in range(n_shards):
        sel = np.nonzero(owner == s)[0]
        local[sel] = np.arange(len(sel))
    gid = local * n_shards + owner
    out = np.full(int(gid.max()) + 1 if len(gid) else 0, -1, dtype=np.int64)
    out[gid] = np.arange(len(owner))
    return out


def slices(n: int, n_shards: int):
    """topic slice boundaries: rank r owns topics [b[r], b[r+1])"""
    return [(d * n) // n_shards for d in range(n_shards + 1)]


def _p(x):
    if x is None:
        return None
    return ctypes.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))


def key_words_for(buf, off):
    """u64 words per order key that cover every topic of a packed batch:
    a topic of n levels needs n <= 32 * words - 1 (kernels.hip key_word)."""
    off = np.asarray(off, dtype=np.int64)
    if len(off) < 2:
        return 1
    b = np.asarray(buf[: int(off[-1])], dtype=np.uint8)
    c = np.zeros(len(b) + 1, dtype=np.int64)
    np.cumsum(b == ord("/"), out=c[1:])
    levels = c[off[1:]] - c[off[:-1]] + 1
    return int(levels.max()) // 32 + 1


class ShardEngine(Engine):
    """The engine of shard `shard` of `n_shards` (one per GPU)."""

    def __init__(self, device, n_shards, shard, filters_hint=0):
        if not 1 <= n_shards <= 8 or not 0 <= shard < n_shards:
            raise ValueError("n_shards must be 1..8 and shard < n_shards")
        super().__init__(device=device, filters_hint=filters_hint)
        self.n_shards, self.shard = n_shards, shard
        # keyed batches of <= 31 levels walk unkeyed; ids take their filter's
        # order key (image.h filter_shape) in the copy-out
        self.set_option("shape_keys", 1)

    def insert_many(self, buf, off):
        """insert the filters of [off[i], off[i+1]) that belong to this shard"""
        n = len(off) - 1
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        return self._check(self.lib.tm_insert_batch_shard(self.h, buf.ctypes.data, off.ctypes.data, n,
                                                          self.n_shards, self.shard), "tm_insert_batch_shard")

    def match_keys_device(self, d_bytes, d_off, n, topic_bytes, d_counts, d_offs, d_ids, d_keys, out_cap, d_total,
                          stream=None, key_words=1):
        """keyed walk; d_keys holds key_words planes of out_cap u64 (word j of
        id i at d_keys[j * out_cap + i])"""
        st = None if stream is None else ctypes.c_void_p(L.stream_handle(stream))
        rc = self.lib.tm_match_batch_device_keys_w(self.h, _p(d_bytes), _p(d_off), n, topic_bytes, _p(d_counts),
                                                   _p(d_offs), _p(d_ids), _p(d_keys), key_words, out_cap,
                                                   _p(d_total), st)
        return self._check(rc, "tm_match_batch_device_keys_w")

    def key_levels(self):
        """most levels of a topic in the last keyed batches (synchronises)"""
        x = ctypes.c_uint32()
        self._check(self.lib.tm_key_levels(self.h, ctypes.byref(x)), "tm_key_levels")
        return x.value

    def merge_device(self, m, d_counts, d_src_base, d_ids, d_keys, d_out_count, d_out_off, d_out_gid, out_cap,
                     d_total, stream=None, key_words=1, key_stride=0):
        st = None if stream is None else ctypes.c_void_p(L.stream_handle(stream))
        rc = self.lib.tm_shard_merge_w(self.h, self.n_shards, m, _p(d_counts), _p(d_src_base), _p(d_ids),
                                       _p(d_keys), key_words, key_stride, _p(d_out_count), _p(d_out_off),
                                       _p(d_out_gid), out_cap, _p(d_total), st)
        return self._check(rc, "tm_shard_merge_w")


def exchange(counts, offs, ids, keys, n, n_shards, rank, group=None, key_words=1, key_stride=0):
    """All-to-all of one rank's keyed lists (torch tensors on the rank's
    device: counts int32[n], offs int64[n+1], ids int32[>= total], keys
    int64[>= total]) so that every rank receives, from every shard, the lists
    of its own topic slice.  Returns (recv_counts int32[S*m] source-major,
    src_base int64[S], recv_ids int32, recv_keys int64, m).  Keys of key_words >
    1 words sit in planes key_stride apart; received keys are planes of the
    received total."""
    import torch
    import torch.distributed as dist
    b = slices(n, n_shards)
    m = b[rank + 1] - b[rank]
    dev = counts.device
    if n_shards == 1:      # one shard: its own lists are the whole result
        return counts[:n], torch.zeros(1, dtype=torch.int64, device=dev), ids, keys, n
    in_splits = [b[d + 1] - b[d] for d in range(n_shards)]
    recv_counts = torch.empty(n_shards * m, dtype=torch.int32, device=dev)
    dist.all_to_all_single(recv_counts, counts[:n].contiguous(), output_split_sizes=[m] * n_shards,
                           input_split_sizes=in_splits, group=group)
    cut = offs[torch.tensor(b, device=dev)].cpu().tolist()     # CSR cut points of the S slices
    send_items = [int(cut[d + 1] - cut[d]) for d in range(n_shards)]
    sizes = torch.tensor(send_items, dtype=torch.int64, device=dev)
    recv_sizes = torch.empty(n_shards, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_sizes, sizes, group=group)
    recv_items = [int(x) for x in recv_sizes.cpu().tolist()]
    tot = sum(recv_items)
    recv_ids = torch.empty(max(tot, 1), dtype=torch.int32, device=dev)
    recv_keys = torch.empty(max(tot, 1) * key_words, dtype=torch.int64, device=dev)
    lo, hi = int(cut[0]), int(cut[-1])
    dist.all_to_all_single(recv_ids[:tot], ids[lo:hi].contiguous(), output_split_sizes=recv_items,
                           input_split_sizes=send_items, group=group)
    for j in range(key_words):
        dist.all_to_all_single(recv_keys[j * tot:(j + 1) * tot], keys[j * key_stride + lo:j * key_stride + hi]
                               .contiguous(), output_split_sizes=recv_items, input_split_sizes=send_items,
                               group=group)
    base = np.zeros(n_shards, dtype=np.int64)
    base[1:] = np.cumsum(recv_items)[:-1]
    src_base = torch.from_numpy(base).to(dev)
    return recv_counts, src_base, recv_ids, recv_keys, m


# ---------------------------------------------------------------------------
# native RCCL exchange (exchange.cpp)

class Comm:
    """one rank's RCCL communicator (tm_comm)"""

    def __init__(self, h, lib):
        self.h, self.lib = h, lib

    @staticmethod
    def unique_id() -> bytes:
        lib = L.load()
        buf = (ctypes.c_uint8 * L.TM_COMM_ID_BYTES)()
        rc = lib.tm_comm_unique_id(buf)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_comm_unique_id")
        return bytes(buf)

    @classmethod
    def init_rank(cls, uid: bytes, nranks: int, rank: int, device: int):
        lib = L.load()
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * L.TM_COMM_ID_BYTES).from_buffer_copy(uid)
        rc = lib.tm_comm_init_rank(buf, nranks, rank, device, ctypes.byref(h))
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_comm_init_rank")
        return cls(h, lib)

    @classmethod
    def init_all(cls, devices):
        lib = L.load()
        n = len(devices)
        hs = (ctypes.c_void_p * n)()
        rc = lib.tm_comm_init_all((ctypes.c_int32 * n)(*devices), n, hs)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_comm_init_all")
        return [cls(ctypes.c_void_p(hs[i]), lib) for i in range(n)]

    @property
    def rccl(self):
        return bool(self.lib.tm_comm_uses_rccl(self.h))

    def set_self_rccl(self, on=True):
        """the rank's own part of every exchange over RCCL too (a one-rank
        communicator then runs the RCCL code paths of the multi-GPU ranks)"""
        rc = self.lib.tm_comm_set_self_rccl(self.h, 1 if on else 0)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_comm_set_self_rccl")

    def close(self):
        if self.h:
            self.lib.tm_comm_destroy(self.h)
            self.h = None


def _xin(n, counts, offs, ids, keys, key_words, key_stride, stream):
    p = lambda x: None if x is None else (x.data_ptr() if hasattr(x, "data_ptr") else int(x))  # noqa: E731
    st = None if stream is None else L.stream_handle(stream)
    return L.TmExchangeIn(n, key_words, p(counts), p(offs), p(ids), p(keys), key_stride, st)


def exchange_native(comm, counts, offs, ids, keys, n, key_words=1, key_stride=0, stream=None):
    """this rank's part of the all-to-all over RCCL; returns the received
    (m, total, d_counts, d_src_base, d_ids, d_keys) device pointers (owned by
    the comm, valid until its next exchange)"""
    xin = _xin(n, counts, offs, ids, keys, key_words, key_stride, stream)
    out = L.TmExchangeOut()
    rc = comm.lib.tm_shard_exchange(comm.h, ctypes.byref(xin), ctypes.byref(out))
    if rc != L.TM_OK:
        raise L.TopicMatchError(rc, "tm_shard_exchange: " + comm.lib.tm_comm_last_error(comm.h).decode())
    return out


class ShardSet:
    """All S shards of one process (one per device in `devices`, repeats
    allowed): the filter set partitioned with tm_shard_of, every batch walked
    by each shard with order keys, exchanged natively (RCCL between distinct
    GPUs, device copies between shards sharing one) and merged per topic slice
    on the slice's GPU.  match_batch returns the merged lists with global ids
    (local * S + shard), in emqx_trie:match/1 order."""

    def __init__(self, devices, filters_hint=0, engines=None):
        """engines: already built ShardEngines (shard s of S on devices[s]),
        e.g. filled in parallel threads; the set takes them over"""
        import torch
        self.torch = torch
        self.devices = list(devices)
        self.S = len(self.devices)
        if engines is not None:
            if len(engines) != self.S or any(e.n_shards != self.S or e.shard != s for s, e in enumerate(engines)):
                raise ValueError("engines must be shards 0..S-1 of S")
            self.engines = list(engines)
        else:
            self.engines = [ShardEngine(d, self.S, s, filters_hint=filters_hint // max(self.S, 1) + 1)
                            for s, d in enumerate(self.devices)]
        self.comms = Comm.init_all(self.devices)

    def insert_many(self, buf, off):
        for e in self.engines:
            e.insert_many(buf, off)
            e.commit()

    def filter_bytes(self, gid: int) -> bytes:
        return self.engines[gid % self.S].filter_bytes(gid // self.S)

    def match_batch(self, tb, to):
        """host batch -> (counts u32[n], offsets u64[n+1], gids u32[total])"""
        torch = self.torch
        S, n = self.S, len(to) - 1
        KW = key_words_for(tb, to)
        lists = []
        # one explicit stream per shard orders walk -> exchange -> merge (the
        # legacy default stream, handle 0, would mean "the engine's stream")
        streams = [torch.cuda.Stream(device=torch.device("cuda", d)) for d in self.devices]
        for s, e in enumerate(self.engines):
            dev = torch.device("cuda", self.devices[s])
            d_b = torch.from_numpy(np.ascontiguousarray(tb).copy()).to(dev)
            d_o = torch.from_numpy(np.ascontiguousarray(to).view(np.int64).copy()).to(dev)
            c = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
            o = torch.empty(n + 1, dtype=torch.int64, device=dev)
            t = torch.zeros(1, dtype=torch.int64, device=dev)
            st = streams[s]
            e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, None, None, 0, t, key_words=KW, stream=st)
            st.synchronize()
            cap = int(t.item()) + 1
            ids = torch.empty(cap, dtype=torch.int32, device=dev)
            keys = torch.empty(cap * KW, dtype=torch.int64, device=dev)
            e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, ids, keys, cap, t, key_words=KW, stream=st)
            st.synchronize()
            check_total(t, cap, "shard %d keyed walk" % s)
            if e.key_levels() > 32 * KW - 1:
                raise RuntimeError("order keys too narrow for the batch")
            lists.append((c, o, ids, keys, cap, d_b, d_o))
        ins = (L.TmExchangeIn * S)(*[_xin(n, c, o, ids, keys, KW, cap, streams[s])
                                     for s, (c, o, ids, keys, cap, _, _) in enumerate(lists)])
        outs = (L.TmExchangeOut * S)()
        hs = (ctypes.c_void_p * S)(*[c.h.value for c in self.comms])
        rc = self.comms[0].lib.tm_shard_exchange_group(hs, S, ins, outs)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_shard_exchange_group: " +
                                    self.comms[0].lib.tm_comm_last_error(self.comms[0].h).decode())
        counts, offs, gids = [], [0], []
        for r in range(S):
            x = outs[r]
            dev = torch.device("cuda", self.devices[r])
            m = x.m
            oc = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
            oo = torch.empty(m + 1, dtype=torch.int64, device=dev)
            tot = torch.zeros(1, dtype=torch.int64, device=dev)
            og = torch.empty(x.total + 1, dtype=torch.int32, device=dev)
            # the merge runs on the comm's stream, after the exchange's copies
            self.engines[r].merge_device(m, x.d_counts, x.d_src_base, x.d_ids, x.d_keys, oc, oo, og, x.total + 1,
                                         tot, stream=streams[r], key_words=KW, key_stride=x.total)
            streams[r].synchronize()
            if check_total(tot, x.total + 1, "merge of slice %d" % r) != x.total:
                raise RuntimeError("merge of slice %d: %d ids merged, %d received" % (r, int(tot.item()), x.total))
            counts.append(oc[:m].cpu().numpy().view(np.uint32))
            offs.extend((oo[1:].cpu().numpy() + offs[-1]).tolist())
            gids.append(og[: x.total].cpu().numpy().view(np.uint32))
        return (np.concatenate(counts) if counts else np.zeros(0, np.uint32), np.asarray(offs, dtype=np.uint64),
                np.concatenate(gids) if gids else np.zeros(0, np.uint32))

    def close(self):
        for c in self.comms:
            c.close()
        for e in self.engines:
            e.close()


# ---------------------------------------------------------------------------
# Routed sharded mode (topicmatch.h tm_route_*; exchange.cpp, route.hip).
#
# Route topic T to the shard of its first `depth` levels, and place filter F
# on the shard of its first `depth` levels when those are all literal, on
# EVERY shard otherwise (a '+' or '#' among them, which can match topics of
# any route).  A filter with literal first levels can only match topics that
# start with the same words (or, shorter than `depth`, exactly its own
# levels), so the owner shard holds every filter that can match T, and its
# walk alone yields emqx_trie:match/1's complete list in order: the order of
# two matching filters is a property of the filters (image.h filter_shape),
# not of the rest of the trie.  No merge, only a topic exchange; filters keep
# global ids on every shard (tm_insert_batch_routed), so the lists need no
# id translation.  The price is the replicated wildcard-led filters.
# tm_route_of hashes the routing key exactly as the device does (route.hip).

def filter_route(filt: bytes, n_shards: int, depth: int = 2) -> int:
    """shard of an (inner, emqx_topic:parse/1-stripped) filter, or -1 = every shard"""
    r = L.load().tm_route_of(filt, len(filt), n_shards, depth, 1)
    return -1 if r == L.TM_ROUTE_ALL else r


def topic_route(topic: bytes, n_shards: int, depth: int = 2) -> int:
    """the shard that owns a publish topic's walk"""
    return L.load().tm_route_of(topic, len(topic), n_shards, depth, 0)


def routed_partition(filters, topics, n_shards: int, depth: int = 2):
    """per-shard filter lists (replicated ones on every shard), topic owners
    and the balance figures: replication factor (filters held over filters),
    topic skew (busiest shard's topics over the mean)"""
    per = [[] for _ in range(n_shards)]
    for f in filters:
        s = filter_route(f, n_shards, depth)
        for d in (range(n_shards) if s < 0 else (s,)):
            per[d].append(f)
    owner = [topic_route(t, n_shards, depth) for t in topics]
    counts = np.bincount(np.asarray(owner, dtype=np.int64), minlength=n_shards)
    stats = {"replication": sum(len(p) for p in per) / max(len(filters), 1),
             "topic_skew": float(counts.max() / max(counts.mean(), 1e-9)),
             "max_shard_filters": max(len(p) for p in per) / max(len(filters), 1)}
    return per, owner, stats


class RoutedEngine(Engine):
    """The engine of routed shard `shard` of `n_shards`: the filters routed to
    it and the replicated ones, under their global ids."""

    def __init__(self, device, n_shards, shard, depth=2, filters_hint=0):
        if not 1 <= n_shards <= 64 or not 0 <= shard < n_shards or depth < 1:
            raise ValueError("n_shards must be 1..64, shard < n_shards, depth >= 1")
        super().__init__(device=device, filters_hint=filters_hint)
        self.n_shards, self.shard, self.depth = n_shards, shard, depth

    def insert_many(self, buf, off, gid_base=0):
        """insert the filters of [off[i], off[i+1]) that live on this shard,
        filter i under global id gid_base + i"""
        n = len(off) - 1
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        return self._check(self.lib.tm_insert_batch_routed(self.h, buf.ctypes.data, off.ctypes.data, n,
                                                           self.n_shards, self.shard, self.depth, gid_base),
                           "tm_insert_batch_routed")


def _sp(stream):
    return None if stream is None else L.stream_handle(stream)


def route_in(n, nbytes, d_bytes, d_off, depth, stream=None):
    return L.TmRouteIn(n, depth, nbytes, _p(d_bytes).value, _p(d_off).value, _sp(stream))


def route_exchange(comm, rin):
    """this rank's topic exchange over RCCL: returns the TmRouteOut of the
    batch it owns (comm-owned device buffers)"""
    out = L.TmRouteOut()
    rc = comm.lib.tm_route_exchange(comm.h, ctypes.byref(rin), ctypes.byref(out))
    if rc != L.TM_OK:
        raise L.TopicMatchError(rc, "tm_route_exchange: " + comm.lib.tm_comm_last_error(comm.h).decode())
    return out


def route_return(comm, counts, offs, ids, stream=None):
    """the owner's lists back to their sources: returns the TmRouteResult of
    this rank's own batch, in its topic order"""
    lists = L.TmRouteLists(_p(counts).value, _p(offs).value, _p(ids).value, _sp(stream))
    res = L.TmRouteResult()
    rc = comm.lib.tm_route_return(comm.h, ctypes.byref(lists), ctypes.byref(res))
    if rc != L.TM_OK:
        raise L.TopicMatchError(rc, "tm_route_return: " + comm.lib.tm_comm_last_error(comm.h).decode())
    return res


class RoutedSet:
    """All S routed shards of one process (one per device in `devices`,
    repeats allowed: shards sharing a GPU exchange by device copies).
    match_batches takes one host batch per shard (each rank's own publishes)
    and returns each batch's lists in its own topic order, with global ids."""

    def __init__(self, devices, depth=2, filters_hint=0):
        import torch
        self.torch = torch
        self.devices = list(devices)
        self.S = len(self.devices)
        self.depth = depth
        self.engines = [RoutedEngine(d, self.S, s, depth=depth, filters_hint=filters_hint)
                        for s, d in enumerate(self.devices)]
        self.comms = Comm.init_all(self.devices)

    def insert_many(self, buf, off, gid_base=0):
        """every shard takes its part of the filter list; the shards build
        in parallel threads (the C-ABI calls release the GIL, each engine has
        its own locks), so S shards of C4's 100M filters build in about one
        shard's time"""
        from concurrent.futures import ThreadPoolExecutor

        def build(e):
            e.insert_many(buf, off, gid_base)
            e.commit()
        with ThreadPoolExecutor(max_workers=min(self.S, 8)) as ex:
            for f in [ex.submit(build, e) for e in self.engines]:
                f.result()

    def match_batches(self, batches):
        """batches: S host batches (tb, to); returns S (counts, offsets, gids)"""
        torch = self.torch
        S = self.S
        lib = self.comms[0].lib
        streams = [torch.cuda.Stream(device=torch.device("cuda", d)) for d in self.devices]
        keep, ins = [], []
        for s, (tb, to) in enumerate(batches):
            dev = torch.device("cuda", self.devices[s])
            pad = np.zeros(len(tb) + 16, dtype=np.uint8)
            pad[:len(tb)] = tb
            d_b = torch.from_numpy(pad).to(dev)
            d_o = torch.from_numpy(np.ascontiguousarray(to).view(np.int64).copy()).to(dev)
            keep.append((d_b, d_o))
            ins.append(route_in(len(to) - 1, int(to[-1] - to[0]), d_b, d_o, self.depth, streams[s]))
        hs = (ctypes.c_void_p * S)(*[c.h.value for c in self.comms])
        outs = (L.TmRouteOut * S)()
        rc = lib.tm_route_exchange_group(hs, S, (L.TmRouteIn * S)(*ins), outs)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_route_exchange_group: " + lib.tm_comm_last_error(self.comms[0].h).decode())
        lists = []
        for s, e in enumerate(self.engines):
            dev = torch.device("cuda", self.devices[s])
            o = outs[s]
            m = o.m
            c = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
            oo = torch.empty(m + 1, dtype=torch.int64, device=dev)
            t = torch.zeros(1, dtype=torch.int64, device=dev)
            e.match_batch_device(o.d_bytes, o.d_off, m, o.bytes, c, oo, None, 0, t, stream=streams[s])
            streams[s].synchronize()
            cap = int(t.item()) + 1
            ids = torch.empty(cap, dtype=torch.int32, device=dev)
            e.match_batch_device(o.d_bytes, o.d_off, m, o.bytes, c, oo, ids, cap, t, stream=streams[s])
            streams[s].synchronize()
            check_total(t, cap, "routed shard %d walk" % s)
            lists.append((c, oo, ids))
        ls = (L.TmRouteLists * S)(*[L.TmRouteLists(_p(c).value, _p(oo).value, _p(ids).value, _sp(streams[s]))
                                    for s, (c, oo, ids) in enumerate(lists)])
        res = (L.TmRouteResult * S)()
        rc = lib.tm_route_return_group(hs, S, ls, res)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_route_return_group: " + lib.tm_comm_last_error(self.comms[0].h).decode())
        out = []
        for s in range(S):
            streams[s].synchronize()
            r = res[s]
            n = r.n
            out.append((_dev_array(r.d_counts, n, np.uint32, self.devices[s]),
                        _dev_array(r.d_offs, n + 1, np.uint64, self.devices[s]),
                        _dev_array(r.d_ids, r.total, np.uint32, self.devices[s])))
        return out

    def close(self):
        for c in self.comms:
            c.close()
        for e in self.engines:
            e.close()


def _dev_array(ptr, n, dtype, device):
    """copy n elements of a device buffer (a raw pointer) to the host"""
    out = np.empty(n, dtype=dtype)
    if n:
        from ._lib import hip_memcpy_d2h
        hip_memcpy_d2h(out.ctypes.data, ptr, out.nbytes, device)
    return out
