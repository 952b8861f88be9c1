"""Batched ACL checks on the GPU (acl.hip) against the oracle
(oracle/pyacl.py): the reference's ACL KATs, then random rule sets x random
credentials / topics (term identity of '', '+', '#', patterns with undefined
or wildcard-looking credentials, v4/v6 CIDRs, nested and/or)."""
import json
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from acl_util import oracle_cred, random_checks, random_rules, rule_term  # noqa: E402
from emqx_amd.emqx_access import AclRules  # noqa: E402
from oracle import pyacl  # noqa: E402

pytestmark = pytest.mark.gpu


def _mirror_cred(c):
    out = dict(c)
    if out.get("peername") is not None:
        out["peername"] = tuple(out["peername"])
    return out


def test_acl_kats_on_device(gpu_device):
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat_acl.json")))
    a = AclRules(gpu_device).load([rule_term(r) for r in kat["suite_rules"]])
    got = a.check_many([_mirror_cred(c) for c, _, _, _ in kat["check_acl"]], [p for _, p, _, _ in kat["check_acl"]],
                       [t for _, _, t, _ in kat["check_acl"]])
    assert [g[0] for g in got] == [w for _, _, _, w in kat["check_acl"]]
    a.close()
    for cred, topic, rule, want in kat["match_rule"]:
        a = AclRules(gpu_device).load([rule_term(rule)])
        acc = rule[2] if len(rule) == 4 and rule[2] != "pubsub" else "publish"
        (res, _), = a.check_many([_mirror_cred(cred)], [acc], [topic])
        assert res == want, (topic, rule)
        a.close()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_acl_random_vs_oracle(gpu_device, seed):
    rng = random.Random(seed)
    rules = random_rules(rng, 40)
    checks = random_checks(rng, 20000)
    a = AclRules(gpu_device).load(rules)
    got = a.check_many([_mirror_cred(c) for c, _, _ in checks], [p for _, p, _ in checks], [t for _, _, t in checks])
    compiled = [pyacl.compile_rule(r) for r in rules]
    hits = 0
    for (cred, pubsub, topic), g in zip(checks, got):
        want = pyacl.check_acl(compiled, oracle_cred(cred), pubsub, topic.encode())
        assert g == want, (cred, pubsub, topic)
        hits += want[0] != "nomatch"
    assert hits > 1000
    a.close()
