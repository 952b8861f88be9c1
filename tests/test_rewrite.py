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


def test_match_regx_replacement_metacharacters():
    """re:replace/4's Replacement (emqx_mod_rewrite.erl:66-68): a captured level
    holding '&' or a backslash is expanded, not copied (OTP re docs; worked by
    hand, parity unpinned: the reference holds no vector for it)"""
    mp = re.compile(rb"^a/(.+)/(.+)$")
    # '&' = the whole match of "\$1", i.e. the text "$1"; the next fold step
    # (I = 2) does not touch it again
    assert match_regx(b"a/b&c/d", mp, b"x/$1/$2") == b"x/b$1c/d"
    # \1: subexpression 1 of the pattern "\$1", which has none: nothing
    assert match_regx(b"a/b\\1c/d", mp, b"x/$1/$2") == b"x/bc/d"
    # \0 is an escaped '0' (re.erl precomp_repl: a backslash before a byte
    # outside 1-9); \g0 and \g{0} are the whole match
    assert match_regx(b"a/b\\0c/d", mp, b"x/$1/$2") == b"x/b0c/d"
    assert match_regx(b"a/b\\g0c/d", mp, b"x/$1/$2") == b"x/b$1c/d"
    assert match_regx(b"a/b\\g{0}c/d", mp, b"x/$1/$2") == b"x/b$1c/d"
    # \& and \\ are the literal characters
    assert match_regx(b"a/b\\&c/d\\\\e", mp, b"$2+$1") == b"d\\e+b&c"
    # "$1" also matches inside "$10" (the fold runs I = 1 first)
    mp10 = re.compile(rb"^" + rb"/".join([rb"(.)"] * 10) + rb"$")
    assert match_regx(b"a/b/c/d/e/f/g/h/i/j", mp10, b"$10|$1") == b"a0|a"
