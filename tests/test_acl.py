"""ACL oracle (oracle/pyacl.py) against the reference's own ACL KATs
(tests/golden/kat_acl.json, test/emqx_access_SUITE.erl), and the ACL rule
builder of the C-ABI on a host-only handle (checks need the GPU: TM_EDEVICE)."""
import json
import os

import pytest

from acl_util import oracle_cred, rule_term
from emqx_amd import _lib
from emqx_amd.emqx_access import AclRules
from oracle import pyacl
from oracle.pytrie import HASH

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def kat():
    return json.load(open(os.path.join(HERE, "golden", "kat_acl.json")))


def test_oracle_check_acl_kats(kat):
    rules = [pyacl.compile_rule(rule_term(r)) for r in kat["suite_rules"]]
    for cred, pubsub, topic, want in kat["check_acl"]:
        got, _ = pyacl.check_acl(rules, oracle_cred(cred), pubsub, topic.encode())
        assert got == want, (cred, pubsub, topic)


def test_oracle_match_rule_kats(kat):
    for cred, topic, rule, want in kat["match_rule"]:
        m = pyacl.match(oracle_cred(cred), topic.encode(), pyacl.compile_rule(rule_term(rule)))
        assert (m if m == "nomatch" else m[1]) == want, (topic, rule)


def test_oracle_compile_rule_kats(kat):
    def w(x):
        return HASH if x == "'#'" else x.encode()
    for rule, filters in kat["compile_rule"]:
        got = pyacl.compile_rule(rule_term(rule))[3]
        want = [pyacl.Pattern([w(x) for x in f["pattern"]]) if isinstance(f, dict) else [w(x) for x in f]
                for f in filters]
        assert len(got) == len(want)
        for g, v in zip(got, want):
            if isinstance(v, pyacl.Pattern):
                assert g == v
            else:
                assert pyacl._weq_list(g, v)


def test_builder_host_only(kat):
    a = AclRules(device=-1).load([rule_term(r) for r in kat["suite_rules"]])
    assert a.lib.tm_acl_rule_count(a.h) == len(kat["suite_rules"])
    with pytest.raises(_lib.TopicMatchError) as e:
        a.check_many([{"client_id": b"c"}], ["publish"], [b"a"])
    assert e.value.code == _lib.TM_EDEVICE
    # malformed builds are refused
    assert a.lib.tm_acl_who(a.h, 0, None, 0, 0) == _lib.TM_EINVAL          # no open rule
    assert a.lib.tm_acl_rule_begin(a.h, 1, 9) == _lib.TM_EINVAL
    a.close()
