"""Projection of the routed sharded mode (emqx_amd/shard.py routed_partition)
at S GPUs from S shard engines measured ONE AT A TIME on one GPU: each shard
holds its literal-led filters plus every wildcard-led one and walks only the
topics it owns.  Projected whole-node rate = batch topics / the slowest
shard's full match time (tokenize + walk + scan + copy-out, HBM-resident
batch).  A projection, not a multi-GPU measurement: no topic exchange is
timed and the shards do not share a node's memory system.

    python tools/bench_routed.py [--config 3] [--shards 8] [--depth 2] [--topics N]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import shard  # noqa: E402
from emqx_amd import workload as W  # noqa: E402
from emqx_amd.engine import Engine, pack  # noqa: E402


def log(*a):
    print("[routed]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--topics", type=int, default=None)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)   # explicit: handle 0 would select the engine's own stream
    cfg = W.CONFIGS[a.config]
    n_topics = a.topics or cfg["topics"]
    t0 = time.time()
    fb, fo = W.filters(a.config)
    tb, to = W.topics(a.config, n=n_topics)
    filters = W.unpack(fb, fo)
    topics = W.unpack(tb, to)
    routes = np.array([shard.filter_route(bytes(f), a.shards, a.depth) for f in filters], dtype=np.int64)
    owner = np.array([shard.topic_route(bytes(t), a.shards, a.depth) for t in topics], dtype=np.int64)
    log("routes of %d filters / %d topics in %.1fs" % (len(filters), len(topics), time.time() - t0))
    res = []
    for s in range(a.shards):
        fsel = np.nonzero((routes == s) | (routes < 0))[0]
        tsel = np.nonzero(owner == s)[0]
        sb, so = pack([bytes(filters[i]) for i in fsel])
        qb, qo = pack([bytes(topics[i]) for i in tsel])
        e = Engine(device=0, filters_hint=len(fsel))
        e.insert_many(sb, so)
        n = len(tsel)
        d_b = torch.from_numpy(qb).to(dev)
        d_o = torch.from_numpy(qo.view(np.int64)).to(dev)
        c = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        o = torch.empty(n + 1, dtype=torch.int64, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        e.match_batch_device(d_b, d_o, n, int(qo[-1]), c, o, None, 0, tot, stream=st)   # sizing pass
        torch.cuda.synchronize(dev)
        cap = int(tot.item()) + 1024
        ids = torch.empty(cap, dtype=torch.int32, device=dev)
        e.match_batch_device(d_b, d_o, n, int(qo[-1]), c, o, ids, cap, tot, stream=st)   # warm-up
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(a.reps):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(st)
            e.match_batch_device(d_b, d_o, n, int(qo[-1]), c, o, ids, cap, tot, stream=st)
            ev1.record(st)
            torch.cuda.synchronize(dev)
            ts.append(ev0.elapsed_time(ev1))
        ms = float(np.median(ts))
        res.append({"shard": s, "filters": int(len(fsel)), "topics": int(n), "ms": ms,
                    "matches": int(tot.item())})
        log("shard %d: %d filters, %d topics, %.3f ms" % (s, len(fsel), n, ms))
        e.close()
        del d_b, d_o, c, o, ids
    slow = max(r["ms"] for r in res)
    print(json.dumps({"config": a.config, "shards": a.shards, "depth": a.depth, "topics": n_topics,
                      "filters": len(filters), "per_shard": res,
                      "filter_share_max": max(r["filters"] for r in res) / len(filters),
                      "slowest_shard_ms": slow,
                      "projected_topics_per_s": n_topics / (slow * 1e-3),
                      "note": "projection: shards measured one at a time on one GPU; no exchange timed"}))


if __name__ == "__main__":
    main()
