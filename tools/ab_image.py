"""Interleaved A/B of image-layout and walk variants on one GPU, one process.

Variants are "opt=val@opt=val..." strings of engine options (tm_set_option).
Options that change the image layout (hot_levels, layout) get their own
engine built from the same filter set; runtime options (split, xcdq,
walk_bpc) are set on that engine before each timing.  Every round times
every variant on the same HBM-resident batch (median and min of the
rounds); the total match count is checked equal across variants.

Run: python tools/ab_image.py --variants "hot_levels=0,hot_levels=0@split=1,hot_levels=4@split=1"
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402

BUILD_OPTS = ("hot_levels", "layout", "hot_edges", "order", "edge_load")


def log(*a):
    print("[ab]", *a, file=sys.stderr, flush=True)


def parse_variant(v):
    opts = {}
    for kv in filter(None, v.split("@")):
        k, x = kv.split("=")
        opts[k] = int(x)
    return opts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=2_000_000)
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    cfg = W.CONFIGS[a.config]
    n_filters = a.filters or cfg["filters"]
    fb, fo = W.filters(a.config, n=n_filters)
    tb, to = W.topics(a.config, n=a.topics)
    n, nbytes = len(to) - 1, int(to[-1])
    variants = {v: parse_variant(v) for v in a.variants.split(",")}
    engines = {}
    for v, opts in variants.items():
        bkey = tuple(sorted((k, x) for k, x in opts.items() if k in BUILD_OPTS))
        if bkey in engines:
            continue
        t0 = time.time()
        e = Engine(device=0, filters_hint=n_filters)
        e.set_option("hot_levels", 4)       # engine default unless the variant says otherwise
        for k, x in bkey:
            e.set_option(k, x)
        e.insert_many(fb, fo)
        e.commit()
        engines[bkey] = e
        log("engine %s built in %.1fs (%d nodes)" % (dict(bkey), time.time() - t0, e.node_count))
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    d_c = torch.empty(n, dtype=torch.int32, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_t = torch.zeros(1, dtype=torch.int64, device=dev)
    first = next(iter(engines.values()))
    first.match_batch_device(d_b, d_o, n, nbytes, d_c, d_oo, None, 0, d_t, stream=st)
    torch.cuda.synchronize(dev)
    total = int(d_t.item())
    cap = total + 1024
    d_i = torch.empty(cap, dtype=torch.int32, device=dev)

    def configure(opts):
        bkey = tuple(sorted((k, x) for k, x in opts.items() if k in BUILD_OPTS))
        e = engines[bkey]
        e.set_option("split", opts.get("split", 1))
        e.set_option("xcdq", opts.get("xcdq", 1))
        e.set_option("walk_bpc", opts.get("walk_bpc", 0))
        e.commit()
        return e

    res = {v: [] for v in variants}
    walk = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v, opts in variants.items():
            e = configure(opts)
            e.match_batch_device(d_b, d_o, n, nbytes, d_c, d_oo, d_i, cap, d_t, stream=st)
            torch.cuda.synchronize(dev)
            e.set_timing(True)
            t1 = time.perf_counter()
            for _ in range(a.reps):
                e.match_batch_device(d_b, d_o, n, nbytes, d_c, d_oo, d_i, cap, d_t, stream=st)
            torch.cuda.synchronize(dev)
            res[v].append((time.perf_counter() - t1) / a.reps * 1e3)
            walk[v].append(e.last_kernel_times().get("walk", 0.0))
            e.set_timing(False)
            assert int(d_t.item()) == total, v
    out = {"config": a.config, "filters": n_filters, "topics": n, "total_ids": total,
           "ms_per_step": {v: {"median": sorted(x)[len(x) // 2], "min": min(x)} for v, x in res.items()},
           "walk_ms": {v: sorted(x)[len(x) // 2] for v, x in walk.items()}}
    for v in variants:
        log("%-40s step %.3f ms (min %.3f)  walk %.3f ms" % (v, out["ms_per_step"][v]["median"],
                                                             out["ms_per_step"][v]["min"], out["walk_ms"][v]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
