"""Subscription churn beside matching (hard part H4).

The reference applies every subscribe/unsubscribe as an emqx_trie insert /
delete inside a mnesia transaction (src/emqx_router.erl:226-231, 252-260);
matches that start after the commit see it.  Here each round applies D
deletes of live filters and D inserts of new ones to the host mirror
(tm_insert / tm_delete: emqx_trie's bookkeeping), commits (tm_commit: waits
for in-flight walks, uploads the dirty 4096-element pages), then matches a
2M-topic HBM-resident batch against the new snapshot.  Reported: deltas/s on
the host, commit time and bytes, match time under churn vs a quiet image,
and a bit-exact check of the final snapshot against O1 rebuilt from the
surviving filter set.

Run: python tools/bench_churn.py [--deltas 100000 --rounds 10]"""
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
    print("[churn]", *a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=2_000_000)
    ap.add_argument("--deltas", type=int, default=100_000, help="inserts and deletes per round (each)")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--check", type=int, default=5_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    cfg = W.CONFIGS[a.config]
    nf = a.filters or cfg["filters"]
    extra = a.deltas * a.rounds
    # one distinct stream of nf + extra filters: the first nf are subscribed
    # up front, the rest arrive as new subscriptions
    fb, fo = W.filters(a.config, n=nf + extra)
    allf = W.unpack(fb, fo)
    e = Engine(device=0, filters_hint=nf + extra)
    e.insert_many(fb, fo[: nf + 1])
    e.commit()
    tb, to = W.topics(a.config, n=a.topics)
    n = len(to) - 1
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    d_c = torch.empty(n, dtype=torch.int32, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_t = torch.zeros(1, dtype=torch.int64, device=dev)
    cap = n * 200
    d_i = torch.empty(cap, dtype=torch.int32, device=dev)

    def match():
        e.match_batch_device(d_b, d_o, n, int(to[-1]), d_c, d_oo, d_i, cap, d_t, stream=st)
        torch.cuda.synchronize(dev)
        assert int(d_t.item()) <= cap

    def timed_match(k=3):
        match()
        t1 = time.perf_counter()
        for _ in range(k):
            match()
        return (time.perf_counter() - t1) / k * 1e3

    quiet_ms = timed_match()
    rng = np.random.default_rng(3)
    live = np.ones(nf + extra, dtype=bool)
    live[nf:] = False
    nxt = nf
    rows = []
    for r in range(a.rounds):
        dels = rng.choice(np.nonzero(live)[0], size=a.deltas, replace=False)
        adds = np.arange(nxt, nxt + a.deltas)
        nxt += a.deltas
        db, do = pack([allf[i] for i in dels])
        ab, ao = pack([allf[i] for i in adds])
        t1 = time.perf_counter()
        e.delete_many(db, do)
        e.insert_many(ab, ao)
        t_apply = time.perf_counter() - t1
        live[dels] = False
        live[adds] = True
        t2 = time.perf_counter()
        e.commit()
        t_commit = time.perf_counter() - t2
        m_ms = timed_match(1)
        rows.append({"apply_s": t_apply, "commit_ms": t_commit * 1e3, "match_ms": m_ms})
        log("round %d: %d deletes + %d inserts applied in %.2fs, commit %.1f ms, match %.2f ms" % (
            r, a.deltas, a.deltas, t_apply, t_commit * 1e3, m_ms))
    churn_ms = timed_match()
    check = None
    if a.check:
        from oracle import O1   # checker only
        surv = [allf[i] for i in np.nonzero(live)[0]]
        o1 = O1(len(surv))
        sb, so = pack(surv)
        o1.insert_many(sb, so)
        topics = W.unpack(tb, to[: a.check + 1])
        got = e.match(topics)
        want = [o1.match(t) for t in topics]
        check = got == want
        log("check of %d topics vs O1 over the %d surviving filters: %s" % (a.check, len(surv), check))
    deltas = 2 * a.deltas * a.rounds
    apply_s = sum(x["apply_s"] for x in rows)
    out = {"workload": "C%d: %d filters, %d rounds of %d deletes + %d inserts, %d-topic batch between rounds" % (
               a.config, nf, a.rounds, a.deltas, a.deltas, n),
           "host_deltas_per_s": deltas / apply_s,
           "commit_ms_median": sorted(x["commit_ms"] for x in rows)[len(rows) // 2],
           "match_ms_quiet": quiet_ms, "match_ms_after_churn": churn_ms,
           "rounds": rows, "filters_live": int(live.sum()), "nodes": e.node_count, "check": check}
    print(json.dumps(out), flush=True)
    e.close()


if __name__ == "__main__":
    main()
