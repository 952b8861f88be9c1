"""Commit while a walk is in flight (engine.cpp Image: two epochs per replica).

A batch queued behind a 3 s spin keeps reading the image it was launched on
while the host deletes / inserts filters and commits.  The batch must see the
old trie and the next one the new trie (each equal to O1's lists); a second
commit, which must reuse the first batch's image, waits for it.

With `require_overlap` the commit must also return before the spin ends.  That
holds only when the engine's stream and the spin's stream sit on different
hardware queues: HIP maps streams onto GPU_MAX_HW_QUEUES queues (4 by
default), and two streams sharing a queue run in order, whatever the API
says.  The GPU test therefore runs this file in a child process with 16
queues and raw HIP streams (torch's stream pool alone is 32 streams).

Run as a script: python tests/inflight_commit.py DEVICE [--overlap]
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from emqx_amd import Engine, pack  # noqa: E402
from emqx_amd import workload as W  # noqa: E402
from oracle import O1  # noqa: E402

SPIN_S = 3.0


def raw_stream(torch, dev):
    """a HIP stream of our own (not from torch's pool), as a torch stream"""
    hip = ctypes.CDLL("libamdhip64.so")
    s = ctypes.c_void_p()
    torch.cuda.set_device(dev)
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0   # hipStreamNonBlocking
    return torch.cuda.ExternalStream(s.value, device=dev)


def run(device, require_overlap):
    import torch
    dev = torch.device("cuda", device)
    fb, fo = W.filters(2, n=200_000)
    tb, to = W.topics(2, n=20_000)
    filters = W.unpack(fb, fo)
    e = Engine(device=device)
    e.insert_many(*pack(filters[:150_000]))
    e.commit()
    n = len(to) - 1
    st = raw_stream(torch, dev)

    # inputs and outputs allocated up front: a pageable H2D copy on st would
    # block the host behind the spin
    d_b = torch.from_numpy(tb.copy()).to(dev)
    d_o = torch.from_numpy(to.view(np.int64).copy()).to(dev)
    bufs = [(torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev),
             torch.empty(4_000_000, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int64, device=dev))
            for _ in range(3)]
    torch.cuda.synchronize(dev)

    def launch():
        c, o, ids, t = bufs.pop()
        e.match_batch_device(d_b, d_o, n, int(to[-1]), c, o, ids, ids.numel(), t, stream=st)
        return c, o, ids, t

    def oracle_lists(live):
        o1 = O1()
        o1.insert_many(*pack([filters[i] for i in live]))
        c, o, i = o1.match_ids(tb, to, threads=8)
        return [[filters[live[j]] for j in i[o[k]:o[k + 1]]] for k in range(n)]

    def host_ids(live):
        """the host API on the live image, pinned to O1 by filter bytes"""
        c, o, ids = e.match_batch(tb, to)
        rows = [[int(x) for x in ids[o[k]:o[k + 1]]] for k in range(n)]
        assert [[e.filter_bytes(x) for x in r] for r in rows] == oracle_lists(live)
        return rows

    def dev_ids(res):
        c, o, ids, t = res
        c, o, ids = c.cpu().numpy().view(np.uint32), o.cpu().numpy().view(np.uint64), ids.cpu().numpy().view(np.uint32)
        assert int(t.item()) == int(o[-1])
        return [[int(x) for x in ids[o[k]:o[k + 1]]] for k in range(n)]

    want0 = host_ids(list(range(150_000)))
    with torch.cuda.stream(st):                 # calibrate the spin kernel's clock
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(st)
        torch.cuda._sleep(100_000_000)
        ev1.record(st)
    ev1.synchronize()
    per_s = 100_000_000 / (ev0.elapsed_time(ev1) / 1e3)
    with torch.cuda.stream(st):
        torch.cuda._sleep(int(per_s * SPIN_S))   # ahead of batch 1
    r1 = launch()
    for f in filters[:20_000]:
        e.delete(f)
    e.insert_many(*pack(filters[150_000:]))
    t0 = time.perf_counter()
    e.commit()
    dt = time.perf_counter() - t0
    overlapped = not st.query()
    want1 = host_ids(list(range(20_000, 200_000)))
    r2 = launch()
    for f in filters[20_000:40_000]:
        e.delete(f)
    e.commit()                                   # writes batch 1's image: waits for it
    want2 = host_ids(list(range(40_000, 200_000)))
    r3 = launch()
    st.synchronize()
    assert dev_ids(r1) == want0
    assert dev_ids(r2) == want1
    assert dev_ids(r3) == want2
    e.close()
    if require_overlap:
        assert overlapped and dt < 1.0, ("the commit took %.2f s and the %.1f s spin had %s: it waited for the "
                                         "walk in flight" % (dt, SPIN_S, "ended" if not overlapped else "not ended"))
    return dt, overlapped


if __name__ == "__main__":
    dt, ov = run(int(sys.argv[1]), "--overlap" in sys.argv)
    print("commit %.4f s, batch still in flight after it: %s" % (dt, ov))
