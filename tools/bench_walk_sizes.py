"""Batch size sweep of the two walks (C3 trie): device-resident batches of n
topics through tm_match_batch_device, the per-lane walk (tm_walk_queue)
against the wave-per-topic walk (tm_walk_wave, option wave_walk_max), mean
ms per batch over repeated launches -- where the wave walk's latency win
turns into a throughput loss sets the default of wave_walk_max.

Run: python tools/bench_walk_sizes.py [--sizes 1024,4096,...]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--sizes", default="256,1024,4096,16384,65536,262144")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    fb, fo = W.filters(a.config)
    e = Engine(device=0)
    e.insert_many(fb, fo)
    e.commit()
    print("[sizes] trie built", file=sys.stderr, flush=True)
    dev = torch.device("cuda", 0)
    st = torch.cuda.Stream(device=dev)
    for n in [int(x) for x in a.sizes.split(",")]:
        tb, to = W.topics(a.config, n=n, stream=7)
        d_b = torch.from_numpy(tb).to(dev)
        d_o = torch.from_numpy(to.view(np.int64)).to(dev)
        c = torch.empty(n, dtype=torch.int32, device=dev)
        oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
        t = torch.zeros(1, dtype=torch.int64, device=dev)
        e.match_batch_device(d_b, d_o, n, int(to[-1]), c, oo, None, 0, t, stream=st)
        torch.cuda.synchronize()
        cap = int(t.item()) + 1024
        ids = torch.empty(cap, dtype=torch.int32, device=dev)
        row = {"topics": n}
        ref = None
        for mode, wmax in (("lane", 0), ("wave", 1 << 30)):
            e.set_option("wave_walk_max", wmax)
            for _ in range(3):
                e.match_batch_device(d_b, d_o, n, int(to[-1]), c, oo, ids, cap, t, stream=st)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                e.match_batch_device(d_b, d_o, n, int(to[-1]), c, oo, ids, cap, t, stream=st)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            got = ids[: int(t.item())].cpu().numpy()
            ref = got if ref is None else ref
            row[mode + "_ms"] = ms
            row[mode + "_topics_per_s"] = n / ms * 1e3
            row[mode + "_same"] = bool(np.array_equal(got, ref))
        print(json.dumps(row), flush=True)
    e.close()


if __name__ == "__main__":
    main()
