"""Debug driver (not product code): the sharded out-of-domain scenario of
tests/test_gpu_shard.py step by step with timestamps, to locate a stall."""
import os
import random
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from emqx_amd import shard  # noqa: E402
from emqx_amd.engine import pack  # noqa: E402

T0 = time.time()


def say(*a):
    print("[%6.2fs]" % (time.time() - T0), *a, flush=True)


shape = int(sys.argv[1]) if len(sys.argv) > 1 else 1
K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rng = random.Random(5)
words = [b"a", b"b", b"+", b"#", b""]
filters = set()
while len(filters) < 1500:   # of ~4,700 possible
    ws = [rng.choice([b"a", b"b", b"c", b"+", b""]) for _ in range(rng.randint(1, 5))]
    if rng.random() < 0.3:
        ws[-1] = b"#"
    filters.add(b"/".join(ws))
filters = sorted(filters)
topics = [b"/".join(rng.choice(words) for _ in range(rng.randint(1, 5))) for _ in range(3000)]
say("scenario built, shape_keys", shape, "K", K)
dev = torch.device("cuda", 0)
fb, fo = pack(filters)
tb, to = pack(topics)
n = len(topics)
d_b = torch.from_numpy(tb).to(dev)
d_o = torch.from_numpy(to.view(np.int64)).to(dev)
e = shard.ShardEngine(0, 1, 0, filters_hint=len(filters))
e.set_option("shape_keys", shape)
e.set_option("stage_k", K)
e.insert_many(fb, fo)
say("engine built")
c = torch.empty(n, dtype=torch.int32, device=dev)
o = torch.empty(n + 1, dtype=torch.int64, device=dev)
tot = torch.zeros(1, dtype=torch.int64, device=dev)
e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, None, None, 0, tot, key_words=1)
say("counting pass launched")
torch.cuda.synchronize()
cap = int(tot.item()) + 16
say("counting pass done, total", cap - 16, "max count", int(c.max().item()))
ids = torch.empty(cap, dtype=torch.int32, device=dev)
keys = torch.empty(cap, dtype=torch.int64, device=dev)
e.match_keys_device(d_b, d_o, n, int(to[-1]), c, o, ids, keys, cap, tot, key_words=1)
say("keyed pass launched")
torch.cuda.synchronize()
say("keyed pass done, total", int(tot.item()))
say("key_levels", e.key_levels())
e.close()
say("closed")
