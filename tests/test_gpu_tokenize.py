"""The device tokenizer (emqx_topic:words/1 + word/1, src/emqx_topic.erl:141-147)
on edge cases, both paths of tm_tokenize: the wave-cooperative one (option
"tok_wave" 1, the default: a wave's topics split into levels, the lanes
take the levels) and the per-lane one (0).  Every topic's list is compared
with O1 id for id, over filters that name each topic's words exactly (so a
wrong word id loses the topic's exact and one-'+' filters).

Cases: empty topics and empty levels ('/', 'a//b', trailing '/'), '$'
topics, the atoms '+' / '#' as levels, bytes that defeat a borrow-based
zero-byte test ('/.' : '.' = '/' ^ 0x01), words of 1-300 bytes (one slot
half, both halves, the arena), 16-64-level topics (levels past the row go
to global memory), waves whose bytes overflow the 4 KiB LDS window and
waves with more than TOK_LMAX (1000) levels (both take the per-lane path
inside the same launch as waves that do not).
"""
import random

import numpy as np
import pytest

from emqx_amd import Engine, pack
from oracle import O1

pytestmark = pytest.mark.gpu


def _topics(rng):
    out = [b"", b"/", b"//", b"a//b", b"a/", b"/a", b"$SYS/x/y", b"$", b"$a/+/#", b"+", b"#", b"a/+/b",
           b"a/#", b"+/+", b"/./", b"a/.b/..c/...", b"./.", b"x" * 255, b"y" * 256, b"z" * 300 + b"/q",
           b"/".join(b"w%d" % i for i in range(16)), b"/".join(b"w%d" % i for i in range(17)),
           b"/".join(b"l%d" % i for i in range(64)), b"/".join([b""] * 40)]
    words = [b"", b".", b"a", b"ab", b"abcdefg", b"abcdefgh", b"abcdefghi", b"0123456789abcdef",
             b"0123456789abcdefg", b"w" * 31, b"k" * 40, b"$x", b"+x", b"x#", b"\x00", b"\x2e\x2f"[:1]]
    for _ in range(3000):
        n = rng.choice([1, 2, 3, 5, 8, 8, 8, 12, 16, 17, 24])
        out.append(b"/".join(rng.choice(words) + (b"%d" % rng.randrange(50) if rng.random() < 0.5 else b"")
                             for _ in range(n)))
    # a run of 64 topics of 20 one-byte levels: 1280 levels in one wave (> TOK_LMAX)
    out += [b"/".join([b"a"] * 20)] * 64
    # a run of 64 topics of 100 bytes: one wave's bytes past the 4 KiB window
    out += [b"/".join([b"m" * 19] * 5)] * 64
    rng.shuffle(out)
    return out


def _filters(topics):
    fs = set()
    for t in topics:
        fs.add(t)
        lv = t.split(b"/")
        for i in range(min(len(lv), 3)):
            fs.add(b"/".join(lv[:i] + [b"+"] + lv[i + 1:]))
        fs.add(b"/".join(lv[:1] + [b"#"]))
    fs.update([b"#", b"+", b"+/#", b"+/+"])
    return sorted(fs)


@pytest.mark.parametrize("tok_wave", [1, 0])
@pytest.mark.parametrize("n_rep", [1, 40])   # 40 x ~3.2K topics: the per-lane queue walk, not the wave walk
def test_tokenizer_edge_cases_vs_o1(gpu_device, tok_wave, n_rep):
    rng = random.Random(11)
    topics = _topics(rng)
    fb, fo = pack(_filters(topics))
    o1 = O1(len(fo))
    o1.insert_many(fb, fo)
    e = Engine(device=gpu_device)
    e.insert_many(fb, fo)
    e.set_option("tok_wave", tok_wave)
    batch = topics * n_rep
    tb, to = pack(batch)
    ec, eo, ei = e.match_batch(tb, to)
    oc, oo, oi = o1.match_ids(tb, to, threads=16)
    assert np.array_equal(ec, oc), [batch[t] for t in np.nonzero(ec != oc)[0][:8]]
    assert np.array_equal(eo, oo) and np.array_equal(ei, oi)
    assert (ec > 0).mean() > 0.95   # nearly every topic meets its own exact filter
    o1.close()
    e.close()
