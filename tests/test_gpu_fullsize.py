"""The headline path checked EXACTLY at its full size (VERDICT r4 "what's
weak" 1): one whole C3 batch -- 10M filters, 8M topics -- under the engine's
default options, every topic's list against O3 (oracle/o3_interned.c,
emqx_trie:match/1 of src/emqx_trie.erl:77-79, 121-145 over interned ids, itself
pinned to O1 and the reference KATs), id for id:

* the device path (tm_match_batch_device, HBM-resident topics: what bench.py
  times) -- at 8M topics the default walk order is the range-local word-hash
  order (presort 5): the range cuts, 32-bit positions and the perm-indexed
  chunk fill at >= 1M-topic XCD ranges run here as they do in the bench;
* the host-buffer path (tm_match_batch_owned) -- at 8M topics the pipelined
  one (option host_pipeline: 1M-topic chunks on two streams).

Long steps print a progress line (capture disabled)."""
import os
import sys
import threading
import time

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

N_TOPICS = 8_000_000


def _say(capsys, t0, msg):
    with capsys.disabled():
        print("[C3-8M %5.0fs] %s" % (time.time() - t0, msg), flush=True)


@pytest.fixture(scope="module")
def c3_full(gpu_device):
    """the C3 engine (defaults), O3 over the same 10M filters, one 8M-topic
    batch and O3's lists of it"""
    from emqx_amd import Engine
    from emqx_amd import workload as W
    from oracle import O3
    fb, fo = W.filters(3)
    tb, to = W.topics(3, n=N_TOPICS, stream=5)
    box, errs = {}, []

    def build_engine():
        try:
            e = Engine(device=gpu_device, filters_hint=10_000_000)
            e.insert_many(fb, fo)
            e.commit()
            box["e"] = e
        except BaseException as x:   # noqa: BLE001
            errs.append(x)

    def build_o3():
        try:
            o = O3(10_000_000)
            o.insert_many(fb, fo)
            th = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count())
            box["want"] = o.match_ids(tb, to, threads=th)
            o.close()
        except BaseException as x:   # noqa: BLE001
            errs.append(x)
    ts = [threading.Thread(target=build_engine), threading.Thread(target=build_o3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]
    yield box["e"], tb, to, box["want"]
    box["e"].close()


def _first_diff(got, want):
    """name the first differing topic (for the failure message)"""
    gc, go, gi = got
    wc, wo, wi = want
    bad = np.flatnonzero(gc != wc)
    if len(bad):
        return "topic %d: count %d, want %d" % (bad[0], gc[bad[0]], wc[bad[0]])
    j = int(np.flatnonzero(gi != wi)[0])
    t = int(np.searchsorted(wo, j, side="right")) - 1
    return "topic %d: ids %s, want %s" % (t, gi[wo[t]:wo[t + 1]].tolist(), wi[wo[t]:wo[t + 1]].tolist())


def _assert_equal(got, want):
    gc, go, gi = got
    wc, wo, wi = want
    ok = len(gc) == len(wc) and np.array_equal(gc, wc) and np.array_equal(go, wo) and np.array_equal(gi, wi)
    assert ok, _first_diff(got, want)


def test_c3_8m_device_default_order_every_topic_equals_o3(gpu_device, c3_full, capsys):
    import torch
    from emqx_amd.engine import check_total
    t0 = time.time()
    e, tb, to, want = c3_full
    n = len(to) - 1
    dev = torch.device("cuda", gpu_device)
    d_b = torch.from_numpy(np.ascontiguousarray(tb)).to(dev)
    d_o = torch.from_numpy(np.ascontiguousarray(to).view(np.int64)).to(dev)
    st = torch.cuda.Stream(device=dev)
    c = torch.empty(n, dtype=torch.int32, device=dev)
    oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    t = torch.zeros(1, dtype=torch.int64, device=dev)
    e.match_batch_device(d_b, d_o, n, int(to[-1]), c, oo, None, 0, t, stream=st)
    st.synchronize()
    # the engine's defaults walk an 8M-topic batch in the range-local
    # word-hash order (option presort 3 -> 5 from sort_min = 1.5M topics)
    assert e.lib.tm_debug_last_order(e.h) == 5
    cap = int(t.item()) + 64
    ids = torch.full((cap,), -1, dtype=torch.int32, device=dev)
    for rep in range(2):   # twice: the second batch runs on the other workspace slot
        e.match_batch_device(d_b, d_o, n, int(to[-1]), c, oo, ids, cap, t, stream=st)
        st.synchronize()
        total = check_total(t, cap, "C3 8M device batch")
        assert e.lib.tm_debug_last_order(e.h) == 5
        got = (c.cpu().numpy().view(np.uint32), oo.cpu().numpy().view(np.uint64),
               ids[:total].cpu().numpy().view(np.uint32))
        _assert_equal(got, want)
        _say(capsys, t0, "device path, pass %d: all %d topics equal O3 (%d ids)" % (rep, n, total))
    assert want[1][-1] > 50 * n   # C3 fan-out ~56


def test_c3_8m_host_pipelined_every_topic_equals_o3(c3_full, capsys):
    t0 = time.time()
    e, tb, to, want = c3_full
    n = len(to) - 1
    got = e.match_batch(tb, to)   # tm_match_batch_owned: pipelined in 1M-topic chunks at 8M
    _assert_equal(got, want)
    _say(capsys, t0, "host pipelined path: all %d topics equal O3" % n)


