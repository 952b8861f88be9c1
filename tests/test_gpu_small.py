"""tm_match_small_device (the micro-batcher's one-launch path, kernels.hip
tm_match_small): every topic's list equals emqx_trie:match/1 (O1) id for id
and in order, read by (offset, count) since lists are placed in completion
order; the lists never overlap and tile [0, total); capacity overflow reports
the exact total and a rerun fills it; topics past the wave's capacity (C5
fan-out, 16+ levels) take the per-lane walk; the kernel's self-resetting
counters survive back-to-back launches on two streams."""
import os

import numpy as np
import pytest

from emqx_amd import Engine, pack
from emqx_amd import workload as W
from oracle import O1

pytestmark = pytest.mark.gpu
L1 = "latin-1"


def _small(e, tb, to, cap=None, stream=None, dev=0):
    """run tm_match_small_device on torch buffers: (counts, offs, ids, total)"""
    import torch
    d = torch.device("cuda", dev)
    n = len(to) - 1
    pad = np.zeros(len(tb) + 16, dtype=np.uint8)
    pad[:len(tb)] = tb
    d_b = torch.from_numpy(pad).to(d)
    d_o = torch.from_numpy(np.ascontiguousarray(to).view(np.int64).copy()).to(d)
    d_c = torch.full((max(n, 1),), -1, dtype=torch.int32, device=d)
    d_oo = torch.full((max(n, 1),), -1, dtype=torch.int64, device=d)
    cap = 64 * n + 1024 if cap is None else cap
    d_i = torch.full((max(cap, 1),), -1, dtype=torch.int32, device=d)
    d_t = torch.full((1,), -1, dtype=torch.int64, device=d)
    torch.cuda.synchronize(d)   # the fills above are on torch's stream; stream=None runs on the engine's
    e.match_small_device(d_b, d_o, n, int(to[-1] - to[0]), d_c, d_oo, d_i, cap, d_t, stream=stream)
    # the whole device: with no stream (or torch's default stream, handle 0)
    # the call runs on the engine's own stream
    torch.cuda.synchronize(d)
    return (d_c.cpu().numpy().view(np.uint32)[:n], d_oo.cpu().numpy().view(np.uint64)[:n],
            d_i.cpu().numpy().view(np.uint32), int(d_t.item()))


def _check(c, o, ids, total, oc, oo, oi):
    n = len(oc)
    assert np.array_equal(c, oc)
    assert total == int(oc.sum())
    # lists tile [0, total) without overlap
    order = np.argsort(o, kind="stable")
    ends = o[order] + c[order].astype(np.uint64)
    assert n == 0 or (o[order][0] == 0 and np.all(o[order][1:] == ends[:-1]) and ends[-1] == total)
    for t in range(n):
        assert np.array_equal(ids[o[t]:o[t] + c[t]], oi[oo[t]:oo[t] + oc[t]]), t


def test_small_c1_equals_o1(gpu_device):
    fb, fo = W.filters(1)
    o1 = O1()
    o1.insert_many(fb, fo)
    e = Engine(device=gpu_device)
    e.insert_many(fb, fo)
    for n in (1, 63, 64, 65, 5000, 30000):
        tb, to = W.topics(1, n=n, stream=n)
        oc, oo, oi = o1.match_ids(tb, to, threads=8)
        _check(*_small(e, tb, to), oc, oo, oi)
    e.close()
    o1.close()


def test_small_golden_vectors(gpu_device, golden):
    """'$' topics vs root wildcards, '#' parents, empty levels, literal '+' /
    '#' levels, long topics (past WREG levels: the per-lane walk)"""
    for vec in golden["o1_vectors"]:
        e = Engine(device=gpu_device)
        fb, fo = pack([f.encode(L1) for f in vec["filters"]])
        e.insert_many(fb, fo)
        tb, to = pack([r["topic"].encode(L1) for r in vec["topics"]])
        c, o, ids, total = _small(e, tb, to)
        for t, row in enumerate(vec["topics"]):
            have = [vec["filters"][int(i)] for i in ids[o[t]:o[t] + c[t]]]
            assert have == row["match"], (vec["name"], row["topic"])
        e.close()


def test_small_capacity_overflow_and_rerun(gpu_device):
    fb, fo = W.filters(1)
    o1 = O1()
    o1.insert_many(fb, fo)
    e = Engine(device=gpu_device)
    e.insert_many(fb, fo)
    tb, to = W.topics(1, n=4000, stream=3)
    oc, oo, oi = o1.match_ids(tb, to, threads=8)
    need = int(oc.sum())
    c, o, ids, total = _small(e, tb, to, cap=need // 3)
    assert total == need and np.array_equal(c, oc)
    for t in range(len(oc)):   # every list placed inside the capacity is complete
        if o[t] + c[t] <= need // 3:
            assert np.array_equal(ids[o[t]:o[t] + c[t]], oi[oo[t]:oo[t] + oc[t]])
    _check(*_small(e, tb, to, cap=total), oc, oo, oi)
    e.close()
    o1.close()


def test_small_c5_fanout_past_the_wave(gpu_device):
    """~900 ids per topic, 16 levels: emissions past the wave's LDS take the
    per-lane walk on lane 0 (count, reserve, emit)"""
    fb, fo = W.filters(5, n=200_000)
    o1 = O1()
    o1.insert_many(fb, fo)
    e = Engine(device=gpu_device)
    e.insert_many(fb, fo)
    tb, to = W.topics(5, n=1500)
    oc, oo, oi = o1.match_ids(tb, to, threads=8)
    _check(*_small(e, tb, to, cap=int(oc.sum()) + 64), oc, oo, oi)
    e.close()
    o1.close()


def test_small_back_to_back_on_two_streams(gpu_device):
    """the per-slot counters reset themselves: many launches in a row, on two
    streams, each exact"""
    import torch
    fb, fo = W.filters(1)
    o1 = O1()
    o1.insert_many(fb, fo)
    e = Engine(device=gpu_device)
    e.insert_many(fb, fo)
    streams = [torch.cuda.Stream(device=torch.device("cuda", gpu_device)) for _ in range(2)]
    for k in range(12):
        tb, to = W.topics(1, n=300 + 97 * k, stream=40 + k)
        oc, oo, oi = o1.match_ids(tb, to, threads=8)
        _check(*_small(e, tb, to, stream=streams[k % 2]), oc, oo, oi)
    # and the CSR path between them still agrees
    tb, to = W.topics(1, n=2000, stream=99)
    hc, ho, hi = e.match_batch(tb, to)
    oc, oo, oi = o1.match_ids(tb, to, threads=8)
    assert np.array_equal(hi, oi) and np.array_equal(hc, oc)
    e.close()
    o1.close()


def test_small_empty_batch(gpu_device):
    e = Engine(device=gpu_device)
    e.insert(b"a/+")
    c, o, ids, total = _small(e, np.zeros(0, dtype=np.uint8), np.zeros(1, dtype=np.uint64))
    assert total == 0
    e.close()
