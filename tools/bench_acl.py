"""Batched ACL checks (f4) on one MI355X: the reference suite's acl.conf rules
plus R generated rules, N checks per call (host buffers in and out).  Reports
checks/s for the whole call and the decision mix; a sample is checked
against the oracle (oracle/pyacl.py).
Run: python tools/bench_acl.py [--checks 1000000 --rules 200]"""
import argparse
import json
import os
import random
import sys
import time

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
    ts = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        got = acl.check_many(creds, subs, topics)
        ts.append(time.perf_counter() - t0)
    from oracle import pyacl   # checker only
    compiled = [pyacl.compile_rule(r) for r in rules]
    ok = all(pyacl.check_acl(compiled, oracle_cred(c), p, t.encode()) == g
             for (c, p, t), g in zip(checks[:5000], got[:5000]))
    mix = {k: sum(1 for g in got if g[0] == k) / len(got) for k in ("allow", "deny", "nomatch")}
    t = sorted(ts)[len(ts) // 2]
    print(json.dumps({"checks": a.checks, "rules": len(rules), "secs": t, "checks_per_s": a.checks / t,
                      "mix": mix, "check": ok,
                      "note": "whole call incl. Python packing of the batch and PCIe copies"}), flush=True)


if __name__ == "__main__":
    main()
