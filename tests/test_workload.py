"""The synthetic workload generator is deterministic and
produces what the configs say.  CPU only."""
import numpy as np

from emqx_amd import workload as W
from emqx_amd import emqx_topic as T


def test_deterministic():
    a = W.filters(1, n=2000)
    b = W.filters(1, n=2000)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    t1 = W.topics(1, n=1000, stream=0)
    t2 = W.topics(1, n=1000, stream=1)
    assert not np.array_equal(t1[0][:100], t2[0][:100])


def test_filters_are_distinct_wildcards():
    buf, off = W.filters(2, n=20000)
    fs = W.unpack(buf, off)
    assert len(set(fs)) == len(fs)
    for f in fs[:5000]:
        assert T.wildcard(f)
        assert 1 <= len(f.split(b"/")) <= 8
        assert T.validate(f)


def test_topics_shape_and_sys_fraction():
    buf, off = W.topics(1, n=20000)
    ts = W.unpack(buf, off)
    assert all(len(t.split(b"/")) == 5 for t in ts)
    sys_n = sum(t.startswith(b"$SYS/") for t in ts)
    assert 100 <= sys_n <= 320                # 1 %
    assert not any(T.wildcard(t) for t in ts[:2000])


def test_c5_share_and_parse():
    buf, off = W.filters(5, n=5000)
    fs = W.unpack(buf, off)
    shared = [f for f in fs if f.startswith(b"$share/")]
    assert 300 <= len(shared) <= 700          # 10 %
    for f in shared[:200]:
        inner, opts = T.parse(f)
        assert "share" in opts and T.wildcard(inner)
    assert max(len(f.split(b"/")) for f in fs) >= 16
