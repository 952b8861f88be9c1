"""Synthetic workloads of SURVEY.md §8(d) (configs C1–C5) through the C
generator emqx_amd/csrc/workload.c (deterministic xoshiro256**, Zipf(1.0)).

Seeds: filters 0xE3A1_0000 + cfg, topics 0xE3A1_1000 + cfg (+ stream offset,
e.g. the rank, so every GPU of a weak-scaling run gets its own batch)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libtmwork.so")


class WkParams(ctypes.Structure):
    _fields_ = [("levels", ctypes.c_uint32), ("share_groups", ctypes.c_uint32),
                ("p_plus", ctypes.c_double), ("p_hash", ctypes.c_double),
                ("sys_frac", ctypes.c_double), ("share_frac", ctypes.c_double),
                ("vocab", ctypes.c_uint32 * 64)]


# SURVEY.md §8(d)
CONFIGS = {
    1: dict(filters=10_000, levels=5, p_plus=0.20, p_hash=0.05, vocab=[4, 16, 64, 256, 1024],
            topics=100_000, sys_frac=0.01, share_frac=0.0),
    2: dict(filters=1_000_000, levels=8, p_plus=0.20, p_hash=0.05, vocab=[8, 32, 128, 512] + [2048] * 4,
            topics=1_000_000, sys_frac=0.0, share_frac=0.0),
    3: dict(filters=10_000_000, levels=8, p_plus=0.20, p_hash=0.05, vocab=[16, 64, 256, 1024] + [4096] * 4,
            topics=8_000_000, sys_frac=0.0, share_frac=0.0),
    4: dict(filters=100_000_000, levels=8, p_plus=0.20, p_hash=0.05, vocab=[32, 128, 512, 2048] + [8192] * 4,
            topics=8_000_000, sys_frac=0.0, share_frac=0.0),
    5: dict(filters=1_000_000, levels=16, p_plus=0.30, p_hash=0.25, vocab=[2 + (i % 3) for i in range(16)],
            topics=1_000_000, sys_frac=0.10, share_frac=0.10),
}

FILTER_SEED = 0xE3A10000
TOPIC_SEED = 0xE3A11000


def _lib():
    if not os.path.exists(_LIB):
        raise ImportError("libtmwork.so not built: run `make`")
    lib = ctypes.CDLL(_LIB)
    lib.wk_generate.restype = ctypes.c_int
    lib.wk_generate.argtypes = [ctypes.POINTER(WkParams), ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64,
                                ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                ctypes.POINTER(ctypes.c_uint64)]
    lib.wk_free.restype = None
    lib.wk_free.argtypes = [ctypes.c_void_p]
    return lib


def params(cfg: int, **over):
    c = dict(CONFIGS[cfg])
    c.update(over)
    p = WkParams()
    p.levels = c["levels"]
    p.share_groups = c.get("share_groups", 8)
    p.p_plus, p.p_hash = c["p_plus"], c["p_hash"]
    p.sys_frac, p.share_frac = c["sys_frac"], c["share_frac"]
    voc = c["vocab"]
    for i in range(p.levels):
        p.vocab[i] = voc[i] if i < len(voc) else voc[-1]
    return p, c


def _gen(p, kind, n, seed, distinct):
    lib = _lib()
    bp, op, nb = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
    rc = lib.wk_generate(ctypes.byref(p), kind, n, seed, 1 if distinct else 0, ctypes.byref(bp), ctypes.byref(op),
                         ctypes.byref(nb))
    if rc != 0:
        raise RuntimeError("wk_generate failed (%d)" % rc)
    try:
        buf = np.ctypeslib.as_array(ctypes.cast(bp, ctypes.POINTER(ctypes.c_uint8)), shape=(nb.value + 8,)).copy()
        off = np.ctypeslib.as_array(ctypes.cast(op, ctypes.POINTER(ctypes.c_uint64)), shape=(n + 1,)).copy()
    finally:
        lib.wk_free(bp)
        lib.wk_free(op)
    return buf, off


def filters(cfg: int, n=None, distinct=True, **over):
    """(bytes u8, offsets u64) of n raw subscription filters of config cfg"""
    p, c = params(cfg, **over)
    n = c["filters"] if n is None else n
    return _gen(p, 0, n, FILTER_SEED + cfg, distinct)


def topics(cfg: int, n=None, stream=0, **over):
    """(bytes u8, offsets u64) of n publish topics of config cfg; `stream`
    selects an independent sequence (e.g. the rank)"""
    p, c = params(cfg, **over)
    n = c["topics"] if n is None else n
    return _gen(p, 1, n, TOPIC_SEED + cfg + (stream << 32), False)


def unpack(buf, off):
    b = buf.tobytes()
    return [b[int(off[i]):int(off[i + 1])] for i in range(len(off) - 1)]
