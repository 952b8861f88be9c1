"""emqx_mod_rewrite's rule choice on the GPU (rewrite.hip) against the
oracle's match/2 transcription (oracle/pytrie.py: rewrite_rule_index) and
the reference's own emqx_topic:match/2 truths (test/emqx_topic_SUITE.erl,
tests/golden/kat_topic.json), which use the binary clause with the '$' rule."""
import os
import random
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


def test_rewrite_topic_suite_kats(gpu_device, golden):
    from emqx_amd.emqx_mod_rewrite import NO_RULE, Rewrite
    from emqx_amd.engine import pack
    for name, filt, want in golden["kat_topic"]["match"]:
        rw = Rewrite([(filt, ".*", "x")], device=gpu_device)
        got = rw.rule_index_batch(*pack([name.encode("latin-1")]))
        assert (got[0] == 0) == want and (want or got[0] == NO_RULE), (name, filt)
        rw.close()


def test_rewrite_first_rule_random_vs_oracle(gpu_device):
    from emqx_amd.emqx_mod_rewrite import NO_RULE, Rewrite
    from emqx_amd.engine import pack
    from oracle import pytrie
    rng = random.Random(17)
    words = [b"a", b"b", b"", b"$SYS", b"c", b"+", b"#", b"+x", b"#y", b"$a"]
    for rep in range(5):
        rules = []
        while len(rules) < rng.randint(1, 40):
            ws = [rng.choice(words) for _ in range(rng.randint(1, 5))]
            rules.append(b"/".join(ws))
        topics = [b"/".join(rng.choice([b"a", b"b", b"", b"$SYS", b"c", b"$a", b"+", b"#"])
                            for _ in range(rng.randint(1, 6))) for _ in range(3000)]
        rw = Rewrite([(f, b"(.*)", b"r/$1") for f in rules], device=gpu_device)
        got = rw.rule_index_batch(*pack(topics))
        for t, g in zip(topics, got):
            w = pytrie.rewrite_rule_index(t, rules)
            assert (NO_RULE if w is None else w) == int(g), (t, rules)
        rw.close()


def test_rewrite_device_api_and_regex(gpu_device):
    import torch
    from emqx_amd.emqx_mod_rewrite import NO_RULE, Rewrite
    from emqx_amd.engine import pack
    # the rules of etc/emqx.conf's module.rewrite examples, in order
    rules = [("x/#", "^x/y/(.+)$", "z/y/$1"), ("y/+/z/#", "^y/(.+)/z/(.+)$", "y/z/$2")]
    rw = Rewrite(rules, device=gpu_device)
    topics = [b"x/y/2", b"x/1/2", b"y/a/z/b", b"y/def", b"$SYS/x", b"x"]
    assert rw.rewrite_many(topics) == [b"z/y/2", b"x/1/2", b"y/z/b", b"y/def", b"$SYS/x", b"x"]
    tb, to = pack(topics)
    dev = torch.device("cuda", gpu_device)
    d_b = torch.from_numpy(tb.copy()).to(dev)
    d_o = torch.from_numpy(to.view(np.int64).copy()).to(dev)
    d_out = torch.empty(len(topics), dtype=torch.int32, device=dev)
    rw.rule_index_device(d_b, d_o, len(topics), d_out)
    torch.cuda.synchronize()
    assert list(d_out.cpu().numpy().view(np.uint32)) == [0, 0, 1, NO_RULE, NO_RULE, 0]
    rw.close()
