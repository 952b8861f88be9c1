"""Subscription churn beside matching (hard part H4).

The reference applies every subscribe / unsubscribe as a route add / del:
emqx_router's handle_cast add_route / del_route (src/emqx_router.erl:153-187)
with the trie bookkeeping of add_trie_route/1 / del_trie_route/1 (:226-260),
inside a mnesia transaction; publishes that start after it see it.

Here every filter is a route (one dest each: a node, or for 1 in 8 a $share
member whose aggre target is its group).  A matcher thread keeps batches of
`--kind` (match: emqx_trie:match/1 ids; routes: match_routes/1; deliveries:
aggre(match_routes/1)) running back to back on its own stream, HBM-resident,
while the main thread applies rounds of D route deletes of live filters and D
route adds of new ones (tm_route_del_batch / tm_route_add_batch: the host
mirror, the trie and the in-place route image) and commits each round
(tm_commit: the dirty pages go to the image epoch no batch reads, then it
flips; walks in flight keep theirs).  Reported: the matcher's topics/s quiet
and under churn, route deltas/s applied on the host, commit latency, and a
check of a topic sample after the last commit against O1 over the surviving
filters (routes: the expected route lists; deliveries: oracle/pytrie.aggre
of them).

Run: python tools/bench_churn.py [--kind routes --deltas 20000 --rounds 10]"""
import argparse
import json
import os
import sys
import threading
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


def dest_of(i):
    """filter i's one route: a node, or (1 in 8) a $share member {Group, Node}"""
    return ("g%d" % (i % 4), "n%d" % (i % 16)) if i % 8 == 0 else "n%d" % (i % 16)


def dest_bytes(d):
    return (d if isinstance(d, str) else "%s|%s" % d).encode()


class Matcher(threading.Thread):
    """batches of one kind back to back on one stream, two in flight"""

    def __init__(self, e, kind, tb, to, dev):
        super().__init__(daemon=True)
        self.e, self.kind, self.dev = e, kind, dev
        self.n = len(to) - 1
        self.nbytes = int(to[-1])
        self.st = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(self.st):
            self.d_b = torch.from_numpy(tb).to(dev)
            self.d_o = torch.from_numpy(to.view(np.int64)).to(dev)
            cap = self.n * 128
            self.cap = cap
            self.outs = [(torch.empty(self.n, dtype=torch.int32, device=dev),
                          torch.empty(self.n + 1, dtype=torch.int64, device=dev),
                          torch.empty(cap, dtype=torch.int32, device=dev),
                          torch.empty(cap if kind != "match" else 1, dtype=torch.int32, device=dev),
                          torch.zeros(1, dtype=torch.int64, device=dev)) for _ in range(2)]
        self.st.synchronize()
        self.stop = threading.Event()
        self.count = 0
        self.error = None

    def launch(self, k):
        c, o, a, b, t = self.outs[k]
        if self.kind == "match":
            self.e.match_batch_device(self.d_b, self.d_o, self.n, self.nbytes, c, o, a, self.cap, t, stream=self.st)
        elif self.kind == "routes":
            self.e.match_routes_batch_device(self.d_b, self.d_o, self.n, self.nbytes, c, o, a, b, self.cap, t,
                                             stream=self.st)
        else:
            self.e.match_deliveries_batch_device(self.d_b, self.d_o, self.n, self.nbytes, c, o, a, b, self.cap, t,
                                                 stream=self.st)

    def run(self):
        try:
            evs = []
            k = 0
            while not self.stop.is_set():
                self.launch(k)
                ev = torch.cuda.Event()
                ev.record(self.st)
                evs.append(ev)
                k ^= 1
                if len(evs) == 2:
                    evs.pop(0).synchronize()
                    self.count += self.n
            for ev in evs:
                ev.synchronize()
                self.count += self.n
        except Exception as ex:   # reported by the main thread
            self.error = ex

    def measure(self, seconds=None, until=None):
        """topics/s while running for `seconds` or until until() returns"""
        self.count = 0
        self.stop.clear()
        t0 = time.perf_counter()
        self.start()
        if until is not None:
            until()
        else:
            time.sleep(seconds)
        self.stop.set()
        self.join()
        dt = time.perf_counter() - t0
        if self.error:
            raise self.error
        torch.cuda.synchronize(self.dev)
        return self.count / dt, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=1_000_000, help="topics per matcher batch")
    ap.add_argument("--kind", choices=["match", "routes", "deliveries"], default="routes")
    ap.add_argument("--deltas", type=int, default=20_000, help="route deletes and adds per round (each)")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--quiet-s", type=float, default=4.0)
    ap.add_argument("--check", type=int, default=2_000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = W.CONFIGS[a.config]
    nf = a.filters or cfg["filters"]
    extra = a.deltas * a.rounds
    fb, fo = W.filters(a.config, n=nf + extra)
    allf = W.unpack(fb, fo)
    dests = [dest_of(i) for i in range(nf + extra)]
    e = Engine(device=0, filters_hint=nf + extra)
    t0 = time.perf_counter()
    if a.kind == "match":
        e.insert_many(fb, fo[: nf + 1])
    else:
        for g in range(4):
            for k in range(16):
                e.dest_target(dest_bytes(("g%d" % g, "n%d" % k)), Engine.TARGET_GROUP, b"g%d" % g)
        db, do = pack([dest_bytes(d) for d in dests[:nf]])
        e.route_add_many(fb, fo[: nf + 1], db, do)
    e.commit()
    log("%d %s built in %.1fs" % (nf, "filters" if a.kind == "match" else "routes", time.perf_counter() - t0))
    tb, to = W.topics(a.config, n=a.topics)
    quiet, _ = Matcher(e, a.kind, tb, to, dev).measure(a.quiet_s)
    log("quiet: %.1fM topics/s" % (quiet / 1e6))

    rng = np.random.default_rng(3)
    live = np.zeros(nf + extra, dtype=bool)
    live[:nf] = True
    rows = []

    def churn():
        nxt = nf
        for r in range(a.rounds):
            dels = rng.choice(np.nonzero(live)[0], size=a.deltas, replace=False)
            adds = np.arange(nxt, nxt + a.deltas)
            nxt += a.deltas
            db, do = pack([allf[i] for i in dels])
            ddb, ddo = pack([dest_bytes(dests[i]) for i in dels])
            ab, ao = pack([allf[i] for i in adds])
            adb, ado = pack([dest_bytes(dests[i]) for i in adds])
            t1 = time.perf_counter()
            if a.kind == "match":
                e.delete_many(db, do)
                e.insert_many(ab, ao)
            else:
                e.route_del_many(db, do, ddb, ddo)
                e.route_add_many(ab, ao, adb, ado)
            t_apply = time.perf_counter() - t1
            live[dels] = False
            live[adds] = True
            t2 = time.perf_counter()
            e.commit()
            t_commit = time.perf_counter() - t2
            rows.append({"apply_ms": t_apply * 1e3, "commit_ms": t_commit * 1e3})
            log("round %d: %d deletes + %d adds applied in %.1f ms, commit %.1f ms" % (
                r, a.deltas, a.deltas, t_apply * 1e3, t_commit * 1e3))

    busy, churn_s = Matcher(e, a.kind, tb, to, dev).measure(until=churn)
    log("under churn: %.1fM topics/s over %.2fs" % (busy / 1e6, churn_s))
    check = None
    if a.check:
        from oracle import O1, pytrie   # checker only
        surv = np.nonzero(live)[0]
        topics = W.unpack(tb, to[: a.check + 1])
        sb, so = pack(topics)
        if a.kind == "match":
            o1 = O1(len(surv))
            o1.insert_many(*pack([allf[i] for i in surv]))
            oc, oo, oi = o1.match_ids(sb, so, threads=8)
            want_f = [[allf[surv[j]] for j in oi[oo[k]:oo[k + 1]]] for k in range(a.check)]
            c, o, ids = e.match_batch(sb, so)
            check = [[e.filter_bytes(int(x)) for x in ids[o[k]:o[k + 1]]] for k in range(a.check)] == want_f
        else:
            # emqx_router: wildcard topics enter the trie, the others are
            # direct routes found by get_routes(Topic) (src/emqx_router.erl:116-118)
            wild = [i for i in surv if pytrie.wildcard(allf[i])]
            direct = {allf[i]: dests[i] for i in surv if not pytrie.wildcard(allf[i])}
            o1 = O1(len(wild))
            o1.insert_many(*pack([allf[i] for i in wild]))
            oc, oo, oi = o1.match_ids(sb, so, threads=8)
            want_r = [([(topics[k], direct[topics[k]])] if topics[k] in direct else []) +
                      [(allf[wild[j]], dests[wild[j]]) for j in oi[oo[k]:oo[k + 1]]] for k in range(a.check)]

            def to_bytes(x, k):
                return topics[k] if int(x) == Engine.TOPIC_ROUTE else e.filter_bytes(int(x))
            if a.kind == "routes":
                c, o, src, dst = e.match_routes_batch(sb, so)
                got = [[(to_bytes(s_, k), e.dest_bytes(int(d)).decode()) for s_, d in
                        zip(src[o[k]:o[k + 1]], dst[o[k]:o[k + 1]])] for k in range(a.check)]
                check = got == [[(f, dest_bytes(d).decode()) for f, d in row] for row in want_r]
            else:
                c, o, to_, tg = e.match_deliveries_batch(sb, so)
                got = [[(to_bytes(x, k), e.target_bytes(int(t))) for x, t in
                        zip(to_[o[k]:o[k] + c[k]], tg[o[k]:o[k] + c[k]])] for k in range(a.check)]
                check = got == [pytrie.aggre(row) for row in want_r]
        log("check of %d topics vs O1 over the %d surviving filters: %s" % (a.check, len(surv), check))
    applied = 2 * a.deltas * a.rounds
    out = {"workload": "C%d: %d filters as routes, %s batches of %d topics back to back on one stream, %d rounds "
                       "of %d route deletes + %d route adds, a commit per round" % (
                           a.config, nf, a.kind, a.topics, a.rounds, a.deltas, a.deltas),
           "kind": a.kind,
           "topics_per_s_quiet": quiet, "topics_per_s_under_churn": busy, "churn_s": churn_s,
           "route_deltas_per_s_host": applied / (sum(x["apply_ms"] for x in rows) / 1e3),
           "route_deltas_per_s_wall": applied / churn_s,
           "commit_ms_median": sorted(x["commit_ms"] for x in rows)[len(rows) // 2],
           "commit_ms_max": max(x["commit_ms"] for x in rows),
           "rounds": rows, "filters_live": int(live.sum()), "check": check}
    print(json.dumps(out), flush=True)
    e.close()


if __name__ == "__main__":
    main()
