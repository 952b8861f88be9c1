"""Batched ACL checks (f4) on one MI355X: the reference suite's acl.conf rules
plus R generated rules, N checks per call (host buffers in and out).  Reports
checks/s three ways -- the whole Python call (packing dominates), packed host
arrays through tm_acl_check_batch (PCIe included), and device-resident through
tm_acl_check_batch_device (HIP events: the kernel) -- and the decision mix; a
sample is checked against the oracle (oracle/pyacl.py).  A rewrite leg times
the batched first-matching-rule kernel (rewrite.hip) the same way.
Run: python tools/bench_acl.py [--checks 1000000 --rules 200]"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from acl_util import oracle_cred, random_checks, random_rules, rule_term  # noqa: E402
from emqx_amd.emqx_access import AclRules  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--checks", type=int, default=1_000_000)
    ap.add_argument("--rules", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rewrite-rules", type=int, default=64, help="rewrite leg: rule count (0 = skip)")
    a = ap.parse_args()
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat_acl.json")))
    rng = random.Random(9)
    rules = random_rules(rng, a.rules) + [rule_term(r) for r in kat["suite_rules"]]
    checks = random_checks(rng, a.checks)
    creds = [dict(c, peername=tuple(c["peername"])) if c.get("peername") else c for c, _, _ in checks]
    subs = [p for _, p, _ in checks]
    topics = [t for _, _, t in checks]
    acl = AclRules(0).load(rules)
    acl.check_many(creds[:1000], subs[:1000], topics[:1000])   # warm-up / upload
    # leg 1: the whole Python call (packing 1M credential dicts dominates)
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        got = acl.check_many(creds, subs, topics)
        ts.append(time.perf_counter() - t0)
    # leg 2: packed host arrays through tm_acl_check_batch (the NIF's shape:
    # packing is the caller's, PCIe copies included)
    arrs = AclRules.pack(creds, subs, topics)
    n = a.checks
    th = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        res, rule = acl.check_packed(n, arrs)
        th.append(time.perf_counter() - t0)
    # leg 3: device-resident batch (tm_acl_check_batch_device), kernel time by
    # HIP events on its stream
    import torch
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    with torch.cuda.stream(st):
        d = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8).reshape(-1)).to(dev) for k, v in arrs.items()}
        d_out = torch.empty(n, dtype=torch.int8, device=dev)
        d_rule = torch.empty(n, dtype=torch.int32, device=dev)
    st.synchronize()
    acl.check_device(n, d, d_out, d_rule, stream=st)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(st)
    for _ in range(a.reps * 3):
        acl.check_device(n, d, d_out, d_rule, stream=st)
    ev[1].record(st)
    ev[1].synchronize()
    dev_ms = ev[0].elapsed_time(ev[1]) / (a.reps * 3)
    same = bool((d_out.cpu().numpy() == res).all() and (d_rule.cpu().numpy().view(np.uint32) == rule).all())
    from oracle import pyacl   # checker only
    compiled = [pyacl.compile_rule(r) for r in rules]
    ok = all(pyacl.check_acl(compiled, oracle_cred(c), p, t.encode()) == g
             for (c, p, t), g in zip(checks[:5000], got[:5000]))
    mix = {k: sum(1 for g in got if g[0] == k) / len(got) for k in ("allow", "deny", "nomatch")}
    t = sorted(ts)[len(ts) // 2]
    thost = sorted(th)[len(th) // 2]
    out = {"checks": n, "rules": len(rules), "mix": mix, "check": ok, "device_equals_host": same,
           "python_call": {"secs": t, "checks_per_s": n / t,
                           "note": "whole Python call incl. packing the credential dicts and PCIe copies"},
           "packed_host_call": {"secs": thost, "checks_per_s": n / thost,
                                "note": "tm_acl_check_batch on packed host arrays: PCIe copies in and out included"},
           "device_resident": {"ms": dev_ms, "checks_per_s": n / (dev_ms / 1e3),
                               "note": "tm_acl_check_batch_device, HIP events on its stream, %d back-to-back calls" %
                                       (a.reps * 3)}}
    if a.rewrite_rules:
        out["rewrite"] = rewrite_leg(a, rng, dev, st)
    print(json.dumps(out), flush=True)


def rewrite_leg(a, rng, dev, st):
    """emqx_mod_rewrite:match_rule/2's rule choice (rewrite.hip) for the same
    number of topics against R rule filters, device-resident, kernel time by
    HIP events; a sample checked against oracle/pytrie.rewrite_rule_index"""
    import torch
    from emqx_amd import workload as W
    from emqx_amd.emqx_mod_rewrite import Rewrite
    from oracle import pytrie   # checker only
    fb, fo = W.filters(3, n=a.rewrite_rules)
    filters = W.unpack(fb, fo)
    rw = Rewrite([(f, b"(.*)", b"x/$1") for f in filters])
    tb, to = W.topics(3, n=a.checks)
    n = len(to) - 1
    with torch.cuda.stream(st):
        d_b = torch.from_numpy(tb.copy()).to(dev)
        d_o = torch.from_numpy(to.view(np.int64).copy()).to(dev)
        d_out = torch.empty(n, dtype=torch.int32, device=dev)
    st.synchronize()
    rw.rule_index_device(d_b, d_o, n, d_out, stream=st)
    import torch.cuda as tc
    ev = [tc.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(st)
    for _ in range(a.reps):
        rw.rule_index_device(d_b, d_o, n, d_out, stream=st)
    ev[1].record(st)
    ev[1].synchronize()
    ms = ev[0].elapsed_time(ev[1]) / a.reps
    got = d_out.cpu().numpy().view(np.uint32)
    topics = W.unpack(tb, to)
    ok = all(pytrie.rewrite_rule_index(topics[i], filters) == (None if got[i] == 0xFFFFFFFF else int(got[i]))
             for i in range(0, n, max(1, n // 3000)))
    hit = float((got != 0xFFFFFFFF).mean())
    rw.close()
    return {"topics": n, "rules": len(filters), "ms": ms, "topics_per_s": n / (ms / 1e3), "hit_rate": hit,
            "check": ok, "note": "tm_rewrite_match_batch_device, one lane per topic scanning the rules in order"}


if __name__ == "__main__":
    main()
