"""Micro-batcher sweep (the NIF's publish path): P producer
threads submit single topics of a C3 batch to tm_batcher_submit, one
completion callback per topic (tools/ubench/batchdrive.cpp), after a warm-up
run; one JSON line per (lanes, max_topics, deadline, producers) point.

Run: python tools/bench_batcher.py [--topics 8000000]"""
import argparse
import ctypes
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--topics", type=int, default=8_000_000)
    ap.add_argument("--lanes", default="2,4")
    ap.add_argument("--max-topics", default="65536,262144")
    ap.add_argument("--deadline-us", default="200")
    ap.add_argument("--producers", default="16")
    ap.add_argument("--cb-threads", default="0")
    ap.add_argument("--eager", default="0", help="comma list of 0/1: TM_BATCHER_EAGER")
    ap.add_argument("--replicas", default="0", help="HIP ordinals of the engine's replicas (repeats: one GPU shared)")
    a = ap.parse_args()
    fb, fo = W.filters(a.config)
    devs = [int(x) for x in a.replicas.split(",")]
    e = Engine(device=devs[0]) if len(devs) == 1 else Engine(devices=devs)
    t0 = time.time()
    e.insert_many(fb, fo)
    e.commit()
    print("[batcher] trie built in %.1fs" % (time.time() - t0), file=sys.stderr)
    tb, to = W.topics(a.config, n=a.topics)
    drv = ctypes.CDLL(os.path.join(ROOT, "tools", "ubench", "libbatchdrive.so"))
    drv.tm_bench_batcher.restype = ctypes.c_int
    drv.tm_bench_batcher.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double)]
    ints = lambda s: [int(x) for x in s.split(",")]  # noqa: E731
    for lanes, mt, dl, prod, cbt, eager in itertools.product(ints(a.lanes), ints(a.max_topics), ints(a.deadline_us),
                                                             ints(a.producers), ints(a.cb_threads), ints(a.eager)):
        print("[batcher] lanes %d, max_topics %d, deadline %d us, producers %d, callback threads %d ..." % (
            lanes, mt, dl, prod, cbt), file=sys.stderr, flush=True)
        res = (ctypes.c_double * 14)()
        rc = drv.tm_bench_batcher(e.h, tb.ctypes.data, to.ctypes.data, len(to) - 1, prod, dl, mt, lanes,
                                  4 if eager else 0, cbt, res)
        print(json.dumps({"replicas": devs, "eager": eager, "lanes": lanes, "max_topics": mt, "deadline_us": dl,
                          "producers": prod,
                          "callback_threads": cbt, "rc": rc,
                          "topics": len(to) - 1, "secs": res[0], "topics_per_s": res[1], "batches": int(res[2]),
                          "mean_batch": res[3], "lat_us_p50": res[4], "lat_us_p99": res[5], "failed": int(res[6]),
                          "matches": int(res[7]),
                          "per_batch_us": {"sealed_to_lane": res[8], "pack": res[9], "device": res[10],
                                           "callbacks": res[11], "device_launch": res[12],
                                           "device_wait": res[13]}}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
