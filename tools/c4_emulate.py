"""Config C4 (100M filters sharded by literal-prefix over 8 GPUs) emulated on ONE
MI355X: the S shard engines are built one after another on the same GPU, each
walks the whole topic batch with order keys (tm_walk_queue<KEYS>), and then
every rank's merge (tm_shard_merge) runs on exactly the lists the all-to-all
would deliver to it.  Times are HIP-event / wall-clock per shard and per rank,
so the 8-GPU step is estimated as

    max_s walk(s)  +  exchange  +  max_r merge(r)

with the exchange priced from the bytes each ordered pair of ranks exchanges
(12 B per id: u32 id + u64 key, plus 4 B per topic count): the 8 GPUs are
fully connected by point-to-point xGMI links (7 per GPU, ~153 GB/s each), so
an all-to-all's pairs move in parallel and the largest pair sets the time.
Only the real 8-GPU run measures it.
A bit-exact check compares the merged lists of the first topics with a
single engine holding the whole filter set when --check > 0.

Run: python tools/c4_emulate.py [--shards 8 --filters 100000000 --topics 8000000]
Writes one JSON line to stdout."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from emqx_amd import shard  # noqa: E402
from emqx_amd import workload as W  # noqa: E402
from emqx_amd.engine import Engine  # noqa: E402

XGMI_LINK_GBS = 153.0   # one xGMI link (7 per GPU, point-to-point; task brief figure)


def log(*a):
    print("[c4]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=None)
    ap.add_argument("--stage-k", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", type=int, default=0, help="topics checked vs one whole-set engine (0 = skip)")
    a = ap.parse_args()
    S = a.shards
    cfg = W.CONFIGS[a.config]
    n_filters = a.filters or cfg["filters"]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    t0 = time.time()
    fb, fo = W.filters(a.config, n=n_filters)
    log("generated %d filters in %.1fs" % (n_filters, time.time() - t0))
    tb, to = W.topics(a.config, n=a.topics or cfg["topics"])
    n = len(to) - 1
    nbytes = int(to[-1])
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    b = shard.slices(n, S)

    res, walk_ms, shard_info = [], [], []
    eng = None
    for s in range(S):
        if eng is not None:
            eng.close()
        t0 = time.time()
        eng = shard.ShardEngine(0, S, s, filters_hint=n_filters // S + 1)
        eng.set_option("stage_k", a.stage_k)
        eng.insert_many(fb, fo)
        eng.commit()
        info = {"filters": eng.filter_count, "nodes": eng.node_count, "image_gb": eng.image_bytes / 1e9,
                "build_s": time.time() - t0}
        c = torch.empty(n, dtype=torch.int32, device=dev)
        o = torch.empty(n + 1, dtype=torch.int64, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        eng.match_keys_device(d_b, d_o, n, nbytes, c, o, None, None, 0, tot, stream=st)
        torch.cuda.synchronize(dev)
        cap = int(tot.item()) + 16
        ids = torch.empty(cap, dtype=torch.int32, device=dev)
        keys = torch.empty(cap, dtype=torch.int64, device=dev)
        eng.match_keys_device(d_b, d_o, n, nbytes, c, o, ids, keys, cap, tot, stream=st)   # warm-up
        torch.cuda.synchronize(dev)
        eng.set_timing(True)
        t1 = time.perf_counter()
        for _ in range(a.reps):
            eng.match_keys_device(d_b, d_o, n, nbytes, c, o, ids, keys, cap, tot, stream=st)
        torch.cuda.synchronize(dev)
        wall = (time.perf_counter() - t1) / a.reps * 1e3
        kms = eng.last_kernel_times()
        eng.set_timing(False)
        info.update(ids=int(tot.item()), step_ms=wall, kernel_ms=kms)
        log("shard %d: %s" % (s, info))
        shard_info.append(info)
        walk_ms.append(wall)
        res.append((c, o, ids, keys))

    # rank r's merge over the lists the all-to-all delivers to it
    merge_ms, recv_bytes, merged = [], [], []
    for r in range(S):
        m = b[r + 1] - b[r]
        rc = torch.cat([res[s][0][b[r]:b[r + 1]] for s in range(S)])
        cuts = [(int(res[s][1][b[r]].item()), int(res[s][1][b[r + 1]].item())) for s in range(S)]
        rid = torch.cat([res[s][2][lo:hi] for s, (lo, hi) in enumerate(cuts)])
        rk = torch.cat([res[s][3][lo:hi] for s, (lo, hi) in enumerate(cuts)])
        sizes = [hi - lo for lo, hi in cuts]
        base = torch.tensor(np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64), device=dev)
        oc = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
        oo = torch.empty(m + 1, dtype=torch.int64, device=dev)
        tot = torch.zeros(1, dtype=torch.int64, device=dev)
        cap = sum(sizes) + 16
        og = torch.empty(cap, dtype=torch.int32, device=dev)
        eng.merge_device(m, rc, base, rid, rk, oc, oo, og, cap, tot, stream=st)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(a.reps):
            eng.merge_device(m, rc, base, rid, rk, oc, oo, og, cap, tot, stream=st)
        torch.cuda.synchronize(dev)
        merge_ms.append((time.perf_counter() - t1) / a.reps * 1e3)
        assert int(tot.item()) == sum(sizes)
        # bytes received from each other shard (own slice stays local)
        recv_bytes.append([12 * sz + 4 * m if s != r else 0 for s, sz in enumerate(sizes)])
        if r == 0:
            merged = (oo[: min(a.check, m) + 1].cpu().numpy().view(np.uint64),
                      og.cpu().numpy().view(np.uint32).astype(np.int64))
    eng.close()

    check_ok = None
    if a.check > 0:
        k = min(a.check, b[1])
        g2i = shard.gid_to_index(shard.shard_of_batch(fb, fo, S), S)
        full = Engine(0, filters_hint=n_filters)
        full.insert_many(fb, fo)
        fc, foff, fid = full.match_batch(tb, to[: k + 1])
        full.close()
        mo, mg = merged
        check_ok = bool(np.array_equal(mo, foff) and np.array_equal(g2i[mg[: int(mo[-1])]], fid.astype(np.int64)))
        log("bit-exact check of %d topics vs the whole-set engine: %s" % (k, check_ok))

    exch_ms = max(max(x) for x in recv_bytes) / (XGMI_LINK_GBS * 1e9) * 1e3
    step_ms = max(walk_ms) + exch_ms + max(merge_ms)
    out = {"workload": "C%d emulated on one MI355X: %d filters sharded over %d GPUs by literal-prefix, %d-topic batch"
                       % (a.config, n_filters, S, n),
           "shards": shard_info, "walk_ms": walk_ms, "merge_ms": merge_ms, "recv_bytes": recv_bytes,
           "exchange_ms_estimate": exch_ms, "exchange_model": "largest pairwise transfer / one xGMI link (%.0f GB/s)"
                                                             % XGMI_LINK_GBS,
           "step_ms_estimate": step_ms, "topics_per_s_estimate": n / (step_ms * 1e-3),
           "check": check_ok}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
