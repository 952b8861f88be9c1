"""ctypes binding of libtopicmatch (include/topicmatch.h).

This is the Python analogue of the reference-side NIF binding
(emqx_amd/csrc/emqx_trie_nif.c).  Loading fails loudly when
the in-tree library has not been built: there is no CPU fallback for the
match path.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libtopicmatch.so")

TM_OK, TM_EINVAL, TM_ENOSPC, TM_EDEVICE, TM_ENOMEM, TM_ENOENT, TM_ERANGE = 0, -1, -2, -3, -4, -5, -6
TM_NO_FILTER = 0xFFFFFFFF
TM_NO_RULE = 0xFFFFFFFF

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)


class TmConfig(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("reserved0", ctypes.c_uint32),
                ("filters_hint", ctypes.c_uint64), ("batch_topics", ctypes.c_uint64),
                ("batch_bytes", ctypes.c_uint64)]


class TmNodeInfo(ctypes.Structure):
    _fields_ = [("edge_count", ctypes.c_uint32), ("filter_id", ctypes.c_uint32)]


class TmBatchStats(ctypes.Structure):
    _fields_ = [("topics", ctypes.c_uint64), ("levels", ctypes.c_uint64),
                ("visits", ctypes.c_uint64), ("edge_reads", ctypes.c_uint64),
                ("matches", ctypes.c_uint64), ("leaf_visits", ctypes.c_uint64),
                ("probe_loads", ctypes.c_uint64), ("prunable_visits", ctypes.c_uint64)]


class TmBatcherConfig(ctypes.Structure):
    _fields_ = [("max_topics", ctypes.c_uint32), ("deadline_us", ctypes.c_uint32), ("max_bytes", ctypes.c_uint64),
                ("flags", ctypes.c_uint32), ("lanes_per_replica", ctypes.c_uint32),
                ("callback_threads", ctypes.c_uint32), ("eager_us", ctypes.c_uint32)]


class TmBatcherStats(ctypes.Structure):
    _fields_ = [(k, ctypes.c_uint64) for k in ("batches", "topics", "results", "max_batch", "size_seals",
                                               "deadline_seals", "failed_batches", "wait_ns", "pack_ns",
                                               "device_ns", "callback_ns", "launch_ns", "sync_ns", "max_wait_ns",
                                               "max_pack_ns", "max_device_ns", "max_callback_ns", "max_sync_ns")]


class TmExchangeIn(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("key_words", ctypes.c_uint32), ("d_counts", ctypes.c_void_p),
                ("d_offs", ctypes.c_void_p), ("d_ids", ctypes.c_void_p), ("d_keys", ctypes.c_void_p),
                ("key_stride", ctypes.c_uint64), ("hip_stream", ctypes.c_void_p)]


class TmExchangeOut(ctypes.Structure):
    _fields_ = [("m", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("total", ctypes.c_uint64),
                ("d_counts", ctypes.c_void_p), ("d_src_base", ctypes.c_void_p), ("d_ids", ctypes.c_void_p),
                ("d_keys", ctypes.c_void_p)]


class TmRouteIn(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("depth", ctypes.c_uint32), ("bytes", ctypes.c_uint64),
                ("d_bytes", ctypes.c_void_p), ("d_off", ctypes.c_void_p), ("hip_stream", ctypes.c_void_p)]


class TmRouteOut(ctypes.Structure):
    _fields_ = [("m", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("bytes", ctypes.c_uint64),
                ("d_bytes", ctypes.c_void_p), ("d_off", ctypes.c_void_p)]


class TmRouteLists(ctypes.Structure):
    _fields_ = [("d_counts", ctypes.c_void_p), ("d_offs", ctypes.c_void_p), ("d_ids", ctypes.c_void_p),
                ("hip_stream", ctypes.c_void_p)]


class TmRouteResult(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("total", ctypes.c_uint64),
                ("d_counts", ctypes.c_void_p), ("d_offs", ctypes.c_void_p), ("d_ids", ctypes.c_void_p)]


TM_ROUTE_ALL = 0xFFFFFFFF
TM_COMM_ID_BYTES = 128
TM_BATCHER_ROUTES = 1
TM_BATCHER_DELIVERIES = 2
TM_BATCHER_EAGER = 4
TM_BATCHER_CSR = 8
TM_BATCHER_STATS_RESET_MAX = 1
DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, c_u32p, c_u32p, ctypes.c_uint32)

# (name, restype, argtypes) — every symbol include/topicmatch.h declares
SIGNATURES = [
    ("tm_open", ctypes.c_int, [ctypes.POINTER(TmConfig), ctypes.POINTER(ctypes.c_void_p)]),
    ("tm_open_devices", ctypes.c_int, [ctypes.POINTER(TmConfig), ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    ("tm_engine_replicas", ctypes.c_int, [ctypes.c_void_p]),
    ("tm_engine_devices", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32]),
    ("tm_close", None, [ctypes.c_void_p]),
    ("tm_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("tm_last_error", ctypes.c_char_p, [ctypes.c_void_p]),
    ("tm_insert", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32]),
    ("tm_insert_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    ("tm_shard_of", ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32]),
    ("tm_shard_of_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_void_p]),
    ("tm_insert_batch_shard",ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_uint32]),
    ("tm_delete", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32]),
    ("tm_delete_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    ("tm_lookup", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(TmNodeInfo)]),
    ("tm_commit", ctypes.c_int, [ctypes.c_void_p, c_u64p]),
    ("tm_engine_device", ctypes.c_int, [ctypes.c_void_p]),
    ("tm_filter_count", ctypes.c_uint64, [ctypes.c_void_p]),
    ("tm_node_count", ctypes.c_uint64, [ctypes.c_void_p]),
    ("tm_image_bytes", ctypes.c_uint64, [ctypes.c_void_p]),
    ("tm_filter_bytes", ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint32, c_u32p]),
    ("tm_filters_gather", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                         ctypes.c_uint64, ctypes.c_void_p]),
    ("tm_dests_gather", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p,
                                       ctypes.c_uint64, ctypes.c_void_p]),
    ("tm_match_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                      c_u64p]),
    ("tm_match_batch_owned", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                            c_u64p]),
    ("tm_free", None, [ctypes.c_void_p]),
    ("tm_match_batch_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    ("tm_match_small_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    ("tm_set_option", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64]),
    ("tm_reserve", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64]),
    ("tm_set_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("tm_match_batch_device_keys", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                   ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                                   ctypes.c_void_p]),
    ("tm_match_batch_device_keys_w", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                                     ctypes.c_void_p]),
    ("tm_key_levels", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    ("tm_shard_merge_w", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    ("tm_shard_merge", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                      ctypes.c_void_p]),
    ("tm_comm_unique_id", ctypes.c_int, [ctypes.c_void_p]),
    ("tm_comm_init_rank", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    ("tm_comm_init_all", ctypes.c_int, [ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32,
                                        ctypes.POINTER(ctypes.c_void_p)]),
    ("tm_comm_destroy", None, [ctypes.c_void_p]),
    ("tm_comm_uses_rccl", ctypes.c_int, [ctypes.c_void_p]),
    ("tm_comm_last_error", ctypes.c_char_p, [ctypes.c_void_p]),
    ("tm_comm_set_self_rccl", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("tm_shard_exchange", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TmExchangeIn),
                                         ctypes.POINTER(TmExchangeOut)]),
    ("tm_shard_exchange_group", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                               ctypes.POINTER(TmExchangeIn), ctypes.POINTER(TmExchangeOut)]),
    ("tm_route_of", ctypes.c_uint32, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_int]),
    ("tm_insert_batch_ids", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                           ctypes.c_void_p]),
    ("tm_insert_batch_routed", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                              ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    ("tm_route_exchange", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TmRouteIn), ctypes.POINTER(TmRouteOut)]),
    ("tm_route_exchange_group", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                               ctypes.POINTER(TmRouteIn), ctypes.POINTER(TmRouteOut)]),
    ("tm_route_return", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TmRouteLists),
                                       ctypes.POINTER(TmRouteResult)]),
    ("tm_route_return_group", ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                             ctypes.POINTER(TmRouteLists), ctypes.POINTER(TmRouteResult)]),
    ("tm_route_add", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                    ctypes.c_uint32]),
    ("tm_route_add_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint32]),
    ("tm_route_del", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                    ctypes.c_uint32]),
    ("tm_route_del_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_uint32]),
    ("tm_lease_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    ("tm_lease_end", None, [ctypes.c_void_p, ctypes.c_uint64]),
    ("tm_route_write", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                      ctypes.c_uint32]),
    ("tm_route_delete_object", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p,
                                              ctypes.c_uint32]),
    ("tm_route_write_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint32]),
    ("tm_get_routes", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_void_p,
                                     ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    ("tm_route_count", ctypes.c_uint64, [ctypes.c_void_p]),
    ("tm_dest_bytes", ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    ("tm_match_routes_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_uint64, ctypes.c_void_p]),
    ("tm_match_routes_batch_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    ("tm_dest_target", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                                      ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]),
    ("tm_target_bytes", ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                          ctypes.POINTER(ctypes.c_uint32)]),
    ("tm_match_deliveries_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                 ctypes.c_void_p]),
    ("tm_match_deliveries_batch_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                        ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p,
                                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                        ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    ("tm_batcher_open", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TmBatcherConfig),
                                       ctypes.POINTER(ctypes.c_void_p)]),
    ("tm_batcher_submit", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32, DONE_FN, ctypes.c_void_p,
                                         c_u64p]),
    ("tm_batcher_flush", ctypes.c_int, [ctypes.c_void_p]),
    ("tm_batcher_get_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TmBatcherStats)]),
    ("tm_batcher_get_stats2", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TmBatcherStats), ctypes.c_uint32,
                                             ctypes.c_uint32]),
    ("tm_batcher_close", None, [ctypes.c_void_p]),
    ("tm_acl_open", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("tm_acl_close", None, [ctypes.c_void_p]),
    ("tm_acl_rule_begin", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32]),
    ("tm_acl_who", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                  ctypes.c_uint32]),
    ("tm_acl_topic", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_uint32]),
    ("tm_acl_rule_end", ctypes.c_int, [ctypes.c_void_p]),
    ("tm_acl_rule_count", ctypes.c_int, [ctypes.c_void_p]),
    ("tm_acl_check_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 13),
    ("tm_acl_check_batch_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.c_void_p] * 14),
    ("tm_rewrite_open", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    ("tm_rewrite_close", None, [ctypes.c_void_p]),
    ("tm_rewrite_rule", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint32]),
    ("tm_rewrite_rule_count", ctypes.c_int, [ctypes.c_void_p]),
    ("tm_rewrite_match_batch", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                              ctypes.c_void_p]),
    ("tm_rewrite_match_batch_device", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                     ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]),
    ("tm_last_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(TmBatchStats)]),
    ("tm_set_timing", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("tm_last_kernel_times", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_char_p),
                                            ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
    ("tm_topic_match", ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]),
    ("tm_topic_wildcard", ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32]),
    ("tm_topic_parse", ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p), c_u32p,
                                      ctypes.POINTER(ctypes.c_void_p), c_u32p]),
    ("tm_build_info", ctypes.c_char_p, []),
]

_lib = None


class TopicMatchError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        super().__init__("%s (%d)%s" % (_strerror(code), code, (": " + msg) if msg else ""))


def _strerror(code):
    try:
        return load().tm_strerror(code).decode()
    except Exception:  # pragma: no cover
        return "status"


def load():
    """Load libtopicmatch.so from the package directory (never from a
    site-packages copy) and bind every exported symbol.  Raises ImportError
    if it was not built — the match path has no fallback."""
    global _lib
    if _lib is not None:
        return _lib
    # torch wheels bundle their own libamdhip64.so.7; when torch is present,
    # load it first so this library binds to the SAME HIP runtime (one HSA
    # context per process, device pointers and streams shared with torch).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError("libtopicmatch.so not built at %s: run `make` (or __graft_entry__.build()); "
                          "the HIP match path has no CPU fallback" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    in_tree = os.path.abspath(LIB_PATH) == os.path.join(_HERE, "libtopicmatch.so")
    for name, res, args in SIGNATURES:
        if not in_tree and not hasattr(lib, name):
            continue   # an older A/B build (bench.py --lib) without a newer entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def hip_memcpy_d2h(dst, src, nbytes, device):
    """synchronous device -> host copy of a raw device pointer (comm-owned
    buffers of the routed exchange), through the HIP runtime the library is
    bound to"""
    lib = load()
    lib.hipSetDevice.argtypes = [ctypes.c_int]
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    if lib.hipSetDevice(device) != 0 or lib.hipMemcpy(dst, src, nbytes, 2) != 0:   # hipMemcpyDeviceToHost
        raise TopicMatchError(TM_EDEVICE, "hipMemcpy device -> host")


def stream_handle(stream):
    """The HIP stream handle of `stream` (a torch stream, an int handle or
    None).  A torch stream first waits for the work already queued on its
    device's current stream -- the fills and copies of the tensors the caller
    just made for this call: torch's side streams are non-blocking, so
    without the wait a zero-fill of an output total could land after the
    engine has written it.  Torch's default stream has handle 0, which the
    C-ABI reads as "the engine's own (non-blocking) stream": that stream
    cannot wait on it, so its queued work is finished on the host first (the
    caller then synchronizes the device before reading the results)."""
    if stream is None or isinstance(stream, int):
        return stream
    import torch
    cur = torch.cuda.current_stream(stream.device)
    if stream.cuda_stream == 0:
        cur.synchronize()
        stream.synchronize()
    elif cur.cuda_stream != stream.cuda_stream:
        stream.wait_stream(cur)
    return stream.cuda_stream
