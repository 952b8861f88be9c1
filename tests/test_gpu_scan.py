"""The CSR offsets of a device batch: tm_scan_single up to 32,768 topics, the
three-launch scan above it (tile sums of 2,048 counts, a scan of the tile
sums, the tiles' offsets).  Batch sizes on either side of the single-launch
bound and of tile edges, 64 and 130 tiles, 600K topics; fan-outs from 0 to
260 ids per topic (past the 128-id stage row) so that tile sums differ
widely.  Counts, offsets and ids must equal O1's exactly.
"""
import random

import numpy as np
import pytest

from emqx_amd import Engine, pack
from oracle import O1

pytestmark = pytest.mark.gpu


HEAVY = [b"h", b"1", b"2", b"3", b"4", b"5", b"6", b"7"]


def _filters():
    fs = {b"#", b"+/#", b"+/+/+"}
    for a in range(40):
        fs.add(b"a%d/#" % a)
        for c in range(8):
            fs.add(b"a%d/+/c%d" % (a, c))
            fs.add(b"a%d/b%d/+" % (a, c))
    for m in range(256):   # every literal / '+' choice over the heavy topic's 8 levels: 256 + 4 matches
        fs.add(b"/".join(b"+" if m >> i & 1 else w for i, w in enumerate(HEAVY)))
    return sorted(fs)


@pytest.mark.parametrize("n", [32768, 32769, 2048 * 64 + 1, 2048 * 130 - 5, 600_001])
def test_offsets_equal_o1(gpu_device, n):
    rng = random.Random(n)
    fb, fo = pack(_filters())
    o1 = O1(len(fo))
    o1.insert_many(fb, fo)
    e = Engine(device=gpu_device)
    e.insert_many(fb, fo)
    pool = [b"a%d/b%d/c%d" % (rng.randrange(45), rng.randrange(10), rng.randrange(10)) for _ in range(500)]
    pool += [b"/".join(HEAVY)] * 3 + [b"zz", b"", b"$SYS/x"]
    batch = [rng.choice(pool) for _ in range(n)]
    tb, to = pack(batch)
    ec, eo, ei = e.match_batch(tb, to)
    oc, oo, oi = o1.match_ids(tb, to, threads=16)
    assert np.array_equal(ec, oc)
    assert np.array_equal(eo, oo), int(np.nonzero(eo != oo)[0][0])
    assert np.array_equal(ei, oi)
    assert ec.max() > 100 and (ec == 0).any()
    o1.close()
    e.close()
