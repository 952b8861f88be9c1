"""emqx_mod_rewrite without a GPU: the oracle's rule choice on the topic
suite's match/2 truths, match_regx/3's capture substitution, and a host-only
rewrite set refusing to match (the rule scan runs on the GPU only)."""
import re

import pytest

from emqx_amd import _lib as L
from emqx_amd.emqx_mod_rewrite import Rewrite, match_regx
from emqx_amd.engine import pack
from oracle import pytrie


def test_oracle_rule_index_on_topic_kats(golden):
    for name, filt, want in golden["kat_topic"]["match"]:
        got = pytrie.rewrite_rule_index(name.encode("latin-1"), [b"zz/never", filt.encode("latin-1")])
        assert (got == 1) == want and got != 0


def test_first_rule_wins_even_on_regex_miss():
    rules = [b"x/#", b"x/y"]
    assert pytrie.rewrite_rule_index(b"x/y", rules) == 0
    assert match_regx(b"x/y", re.compile(b"^q/(.+)$"), b"z/$1") == b"x/y"
    assert match_regx(b"a/b/c", re.compile(b"^a/(.+)/(.+)$"), b"$2/$1/$2") == b"c/b/c"


def test_host_only_rewrite_refuses():
    rw = Rewrite([("a/#", "(.*)", "b")], device=-1)
    with pytest.raises(L.TopicMatchError) as ex:
        rw.rule_index_batch(*pack([b"a/b"]))
    assert ex.value.code == L.TM_EDEVICE
    rw.close()
