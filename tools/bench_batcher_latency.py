"""Micro-batcher latency under offered load.

The reference answers every publish synchronously inside the publisher's
process (src/emqx_broker.erl:148-157); behind the NIF a publish waits for its
micro-batch.  This drives the batcher open-loop (tools/ubench/batchdrive.cpp
tm_bench_batcher_open_loop): 16 producer threads submit single C3 topics at a
fixed aggregate rate, and the latency of a publish is its callback time minus
its SCHEDULED time (a producer that falls behind is charged, as a publisher
kept waiting would be).  One JSON line per (rate, deadline) point.

Run: python tools/bench_batcher_latency.py [--rates 1e6,1e7,5e7,1e8] [--deadlines 50,100,200]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402


def log(*a):
    print("[latency]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--topics", type=int, default=4_000_000, help="distinct topics cycled by the producers")
    ap.add_argument("--rates", default="1e6,1e7,5e7,1e8")
    ap.add_argument("--deadlines", default="50,100,200")
    ap.add_argument("--seconds", type=float, default=0.5, help="offered-load duration per point")
    ap.add_argument("--max-topics", type=int, default=262144)
    ap.add_argument("--lanes", type=int, default=4)
    ap.add_argument("--cb-threads", type=int, default=8)
    ap.add_argument("--producers", type=int, default=16)
    ap.add_argument("--opt", action="append", default=[], help="engine option name=value (repeatable)")
    ap.add_argument("--lib", default=None, help="EXPERIMENT: alternative build of libtopicmatch.so")
    ap.add_argument("--eager", default="0", help="comma list of 0/1: TM_BATCHER_EAGER (seal when a lane is free)")
    ap.add_argument("--eager-us", default="0", help="comma list: tm_batcher_config.eager_us (0 = the library's "
                    "default) for the eager points")
    ap.add_argument("--csr", default="0", help="comma list of 0/1: TM_BATCHER_CSR (small batches through the "
                    "four-launch CSR path instead of the one-launch tm_match_small_device)")
    a = ap.parse_args()
    if a.lib:
        from emqx_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    fb, fo = W.filters(a.config)
    e = Engine(device=0)
    for kv in a.opt:
        k, x = kv.split("=")
        e.set_option(k, int(x))
    t0 = time.time()
    e.insert_many(fb, fo)
    e.commit()
    log("trie built in %.1fs" % (time.time() - t0))
    tb, to = W.topics(a.config, n=a.topics)
    drv = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "libbatchdrive.so"))
    f = drv.tm_bench_batcher_open_loop
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_double,
                  ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.c_uint32, ctypes.POINTER(ctypes.c_double)]
    for rate, eager, csr, eus in [(float(x), int(g), int(c), int(u)) for x in a.rates.split(",")
                                  for g in a.eager.split(",") for c in a.csr.split(",")
                                  for u in (a.eager_us.split(",") if int(g) else ["0"])]:
        for dl in [int(x) for x in a.deadlines.split(",")]:
            total = max(100_000, int(rate * a.seconds))
            log("offered %.0fM publishes/s, deadline %d us, %d publishes ..." % (rate / 1e6, dl, total))
            r = (ctypes.c_double * 24)()
            rc = f(e.h, tb.ctypes.data, to.ctypes.data, len(to) - 1, a.producers, rate, total, dl, a.max_topics,
                   a.lanes, (4 if eager else 0) | (8 if csr else 0) | (eus << 16), a.cb_threads, r)
            print(json.dumps({"opts": a.opt, "eager": eager, "eager_us": eus, "csr": csr, "offered_per_s": rate, "deadline_us": dl, "max_topics": a.max_topics,
                              "lanes": a.lanes, "callback_threads": a.cb_threads, "producers": a.producers,
                              "rc": rc, "publishes": total, "secs": r[0], "achieved_per_s": r[1],
                              "batches": int(r[2]), "mean_batch": r[3], "lat_us_p50": r[4], "lat_us_p99": r[5],
                              "lat_us_p999": r[6], "lat_us_max": r[7], "failed": int(r[8]),
                              "max_producer_lag_us": r[9],
                              "per_batch_us": {"sealed_to_lane": r[10], "pack": r[11], "device": r[12],
                                               "callbacks": r[13], "device_launch": r[14],
                                               "device_wait": r[15]},
                              "worst_batch_us": {"sealed_to_lane": r[16], "pack": r[17], "device": r[18],
                                                 "callbacks": r[19], "device_wait": r[20]}}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
