"""The N>1 control plane on CPU: two gloo ranks run the bench's timed region
(barrier, per-rank steps, max over ranks) and its per-rank topic streams.
The data path has no collective (replicated trie, topic-sharded batches)."""
import os
import socket
import sys

import numpy as np  # noqa: F401
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import workload as W  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import time

    import torch.distributed as dist
    from emqx_amd import multi
    from emqx_amd import workload as W
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r, w, lr = multi.env_rank()
    # each rank's step sleeps a different time: the reported time is the max
    delay = 0.02 * (rank + 1)
    dt = multi.timed_region(lambda: time.sleep(delay), 3, lambda: None)
    tb, to = W.topics(1, n=500, stream=multi.topic_stream(r))
    # parity_check is the AND over ranks: one failing rank fails the line
    and_all = multi.all_true(True)
    and_one = multi.all_true(rank == 0)
    # strong scaling (bench.py's default): rank r walks slice r of the batch
    import argparse
    sys.path.insert(0, ROOT)
    import bench
    a = argparse.Namespace(batches=2, scaling="strong", topics=1001, config=1, presort=None)
    sl = [(tb_.tobytes()[:int(to_[-1])], to_.tolist()) for tb_, to_ in bench.make_batches(a, None, r, w)]
    q.put((rank, r, w, dt, tb[:int(to[-1])].tobytes(), and_all, and_one, sl))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_timed_region_and_streams(world):
    """world 2, and world 8 (the driver's 8-GPU launch, rehearsed on the CPU:
    the 8-rank GPU run itself is the driver's): every rank's step time is the
    max over ranks, parity is the AND over ranks, the strong slices of every
    batch are the whole batch in rank order, and the ranks' own (weak)
    topic streams differ"""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [x[1] for x in res] == list(range(world)) and all(x[2] == world for x in res)
    assert all(x[5] for x in res) and not any(x[6] for x in res)   # AND over ranks
    for b in range(2):   # the ranks' strong slices are the whole batch, in order
        tb, to = W.topics(1, n=1001, stream=b)
        whole = [bytes(tb[int(to[i]):int(to[i + 1])]) for i in range(1001)]
        got = []
        for x in res:
            bb, oo = x[7][b]
            got += [bb[oo[i]:oo[i + 1]] for i in range(len(oo) - 1)]
        assert got == whole
        assert max(len(x[7][b][1]) - 1 for x in res) - min(len(x[7][b][1]) - 1 for x in res) <= 1
    dts = [x[3] for x in res]
    assert max(dts) - min(dts) < 1e-9          # every rank reports the same max
    assert dts[0] >= 3 * 0.02 * world          # the slowest rank's time
    assert len(set(x[4] for x in res)) == world   # independent topic streams
