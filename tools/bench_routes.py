"""emqx_router:match_routes/1 and emqx_broker:aggre/1 over it on one MI355X at
C3 scale.

Route table: every one of the 10M C3 wildcard filters routes to one of 8
nodes, every 4th filter also to a shared-subscription dest {Group, Node};
1M publish topics carry a direct (exact-topic) route.  One step = the whole
match_routes/1 path of a 2M-topic HBM-resident batch: tokenizer, trie walk,
CSR emission, route count / scan / emit (routes.hip).  Timed beside the
trie-only step (emqx_trie:match/1) and the deliveries step (aggre(match_routes
(T)), aggre.hip after the route kernels) on the same batch, interleaved.

Run: python tools/bench_routes.py [--filters N --topics N --steps K]
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

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402
from emqx_amd.engine import pack  # noqa: E402


def log(*a):
    print("[routes]", *a, file=sys.stderr, flush=True)


def fixed_dests(idx, names):
    """packed dest bytes for route i = names[idx[i]] (equal-length names)"""
    table = np.frombuffer(b"".join(names), dtype=np.uint8).reshape(len(names), -1)
    w = table.shape[1]
    buf = np.concatenate([table[idx].ravel(), np.zeros(8, dtype=np.uint8)])
    off = np.arange(len(idx) + 1, dtype=np.uint64) * np.uint64(w)
    return buf, off


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=2_000_000)
    ap.add_argument("--exact", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--check", type=int, default=20_000)
    ap.add_argument("--lib", default=None, help="EXPERIMENT: alternative build of libtopicmatch.so (A/B)")
    a = ap.parse_args()
    if a.lib:
        from emqx_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    cfg = W.CONFIGS[a.config]
    nf = a.filters or cfg["filters"]
    t0 = time.time()
    fb, fo = W.filters(a.config, n=nf)
    e = Engine(device=0, filters_hint=nf)
    nodes = [b"emqx@node%02d" % k for k in range(8)]
    groups = [b"g%02d|emqx@node%02d" % (k, k) for k in range(8)]
    db, do = fixed_dests(np.arange(nf) % 8, nodes)
    e.route_add_many(fb, fo, db, do)
    sub = W.unpack(fb, fo)[::4]
    sb, so = pack(sub)
    db, do = fixed_dests(np.arange(len(sub)) % 8, groups)
    e.route_add_many(sb, so, db, do)
    del sub, sb, so
    xb, xo = W.topics(a.config, n=a.exact, stream=99)
    db, do = fixed_dests(np.zeros(a.exact, dtype=np.int64), nodes)
    e.route_add_many(xb, xo, db, do)
    for k in range(8):   # aggre targets: node atoms and $share groups
        e.dest_target(nodes[k], Engine.TARGET_NODE, nodes[k])
        e.dest_target(groups[k], Engine.TARGET_GROUP, groups[k].split(b"|")[0])
    e.commit()
    log("routes: %d over %d filters + %d exact topics, built in %.1fs" % (e.route_count, e.filter_count, a.exact,
                                                                          time.time() - t0))

    tb, to = W.topics(a.config, n=a.topics)
    # a share of the batch hits the exact routes: publish to topics that have direct routes
    n = len(to) - 1
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    d_c = torch.empty(n, dtype=torch.int32, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_t = torch.zeros(1, dtype=torch.int64, device=dev)
    e.match_routes_batch_device(d_b, d_o, n, int(to[-1]), d_c, d_oo, None, None, 0, d_t, stream=st)
    torch.cuda.synchronize(dev)
    rtotal = int(d_t.item())
    cap = rtotal + 1024
    d_s = torch.empty(cap, dtype=torch.int32, device=dev)
    d_d = torch.empty(cap, dtype=torch.int32, device=dev)
    ic = torch.empty(n, dtype=torch.int32, device=dev)
    io = torch.empty(n + 1, dtype=torch.int64, device=dev)
    it = torch.zeros(1, dtype=torch.int64, device=dev)
    e.match_batch_device(d_b, d_o, n, int(to[-1]), ic, io, None, 0, it, stream=st)
    torch.cuda.synchronize(dev)
    itotal = int(it.item())
    d_i = torch.empty(itotal + 1024, dtype=torch.int32, device=dev)

    d_ac = torch.empty(n, dtype=torch.int32, device=dev)
    d_ao = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_at = torch.empty(cap, dtype=torch.int32, device=dev)
    d_ag = torch.empty(cap, dtype=torch.int32, device=dev)
    d_atot = torch.zeros(1, dtype=torch.int64, device=dev)

    def deliveries_step():
        e.match_deliveries_batch_device(d_b, d_o, n, int(to[-1]), d_ac, d_ao, d_at, d_ag, cap, d_atot, stream=st)

    def routes_step():
        e.match_routes_batch_device(d_b, d_o, n, int(to[-1]), d_c, d_oo, d_s, d_d, cap, d_t, stream=st)

    def trie_step():
        e.match_batch_device(d_b, d_o, n, int(to[-1]), ic, io, d_i, itotal + 1024, it, stream=st)

    res = {"match_routes": [], "trie_match": [], "deliveries": []}
    for _ in range(3):
        for name, fn in (("match_routes", routes_step), ("trie_match", trie_step), ("deliveries", deliveries_step)):
            fn()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            for _ in range(a.steps):
                fn()
            torch.cuda.synchronize(dev)
            res[name].append((time.perf_counter() - t1) / a.steps * 1e3)
    assert int(d_t.item()) == rtotal
    ms = {k: sorted(v)[len(v) // 2] for k, v in res.items()}

    check = None
    if a.check:
        from oracle import O1   # checker only: route expansion of O1's ordered ids on the host
        k = min(a.check, n)
        o1 = O1(nf)
        o1.insert_many(fb, fo)
        oc, oo, oi = o1.match_ids(tb, to[: k + 1], threads=16)
        exact = set(W.unpack(xb, xo))
        topics = W.unpack(tb, to[: k + 1])
        src = d_s.cpu().numpy().view(np.uint32)
        dst = d_d.cpu().numpy().view(np.uint32)
        off = d_oo[: k + 1].cpu().numpy().view(np.uint64)
        names = [e.dest_bytes(i) for i in range(len(nodes) + len(groups))]
        ok = True
        for t in range(k):
            want = [(0xFFFFFFFF, nodes[0])] if topics[t] in exact else []
            for fid in oi[int(oo[t]):int(oo[t + 1])]:
                fid = int(fid)
                want.append((fid, nodes[fid % 8]))
                if fid % 4 == 0:
                    want.append((fid, groups[(fid // 4) % 8]))
            got = [(int(src[j]), names[int(dst[j])]) for j in range(int(off[t]), int(off[t + 1]))]
            if got != want:
                ok = False
                log("mismatch at topic %d: %s vs %s" % (t, got[:6], want[:6]))
                break
        log("check of %d topics vs O1 + host route expansion: %s" % (k, ok))
        # aggre(match_routes(T)) vs the oracle's transcription of aggre/1
        from oracle.pytrie import aggre
        ka = min(k, 5000)
        at = d_at.cpu().numpy().view(np.uint32)
        ag = d_ag.cpu().numpy().view(np.uint32)
        ao = d_ao[: ka + 1].cpu().numpy().view(np.uint64)
        ac = d_ac[:ka].cpu().numpy().view(np.uint32)
        fcache, tcache = {}, {}

        def fname(fid):
            if fid not in fcache:
                fcache[fid] = e.filter_bytes(fid)
            return fcache[fid]
        for t in range(ka):
            rl = [(topics[t], nodes[0])] if topics[t] in exact else []
            for fid in oi[int(oo[t]):int(oo[t + 1])]:
                fid = int(fid)
                rl.append((fname(fid), nodes[fid % 8]))
                if fid % 4 == 0:
                    g = groups[(fid // 4) % 8].split(b"|")
                    rl.append((fname(fid), (g[0], g[1])))
            got = []
            for j in range(int(ao[t]), int(ao[t]) + int(ac[t])):
                g = int(ag[j])
                if g not in tcache:
                    tcache[g] = e.target_bytes(g)
                got.append((topics[t] if int(at[j]) == 0xFFFFFFFF else fname(int(at[j])), tcache[g]))
            if got != aggre(rl):
                ok = False
                log("aggre mismatch at topic %d: %s vs %s" % (t, got[:6], aggre(rl)[:6]))
                break
        log("aggre check of %d topics vs oracle aggre/1: %s" % (ka, ok))
        check = ok
    out = {"workload": "C%d: %d filters, %d routes (%d exact topics), %d-topic batch" % (
               a.config, nf, e.route_count, a.exact, n),
           "ms_per_step": ms, "topics_per_s": {k: n / (v * 1e-3) for k, v in ms.items()},
           "routes_per_topic": rtotal / n, "routes_per_s": rtotal / (ms["match_routes"] * 1e-3),
           "route_expansion_ms": ms["match_routes"] - ms["trie_match"],
           "deliveries_per_topic": int(d_ac.view(torch.int32).sum().item()) / n, "aggre_ms": ms["deliveries"] - ms["match_routes"],
           "check": check}
    print(json.dumps(out), flush=True)
    e.close()


if __name__ == "__main__":
    main()
