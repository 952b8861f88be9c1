"""Diagnostic: first mismatching topic of the C5 sample (GPU vs O1)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from emqx_amd import Engine, emqx_topic as T  # noqa: E402
from emqx_amd import workload as W  # noqa: E402
from emqx_amd.engine import pack  # noqa: E402
from oracle import O1  # noqa: E402
from emqx_amd import _lib  # noqa: E402

if len(sys.argv) > 1:   # alternative build of libtopicmatch.so (bisecting)
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])

fb, fo = W.filters(5, n=200_000)
inner = [T.parse(f)[0] for f in W.unpack(fb, fo)]
ib, io = pack(inner)
o1 = O1(len(io))
o1.insert_many(ib, io)
for k in [512]:
    e = Engine(device=0, filters_hint=len(io) - 1)
    e.set_option("stage_k", k)
    e.insert_many(ib, io)
    tb, to = W.topics(5, n=5000)
    ec, eo, ei = e.match_batch(tb, to)
    oc, oo, oi = o1.match_ids(tb, to, threads=16)
    bad = 0
    for t in range(len(ec)):
        a = ei[int(eo[t]):int(eo[t]) + int(ec[t])]
        b = oi[int(oo[t]):int(oo[t]) + int(oc[t])]
        if not np.array_equal(a, b):
            bad += 1
            if bad <= 3:
                d = np.nonzero(a != b)[0]
                print("K=%d topic %d count %d mismatches %d first at %s: got %s want %s; set-equal %s" % (
                    k, t, ec[t], len(d), d[:5], a[d[:5]], b[d[:5]], sorted(a) == sorted(b)))
    print("K=%d: %d of %d topics differ; counts equal %s" % (k, bad, len(ec), np.array_equal(ec, oc)))
    e.close()
