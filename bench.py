"""bench.py — topic matches/sec at 10M wildcard filters on MI355X.

One step = one batch of publish topics (bytes + offsets already resident in
HBM) through the whole hot path of emqx_trie:match/1: device tokenizer
(emqx_topic:words/1), NFA walk, CSR emission of the ordered match lists.

Workload: 10M distinct wildcard filters (8 levels max,
p+ 0.20, p# 0.05, Zipf(1.0) words over 16/64/256/1024/4096x4), replicated on
every GPU; each rank matches its own batch of 8-level topics (weak scaling,
no collective on the data path).  `value` = topics matched per second over all
ranks (max-over-ranks step time).

Run: python bench.py [--gpus N --steps K --warmup W]
     torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import multi  # noqa: E402
from emqx_amd import workload as W  # noqa: E402

METRIC = "topic matches/sec (whole node) at 10M wildcard filters; % HBM roofline"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3, help="SURVEY §8(d) config (3 = the metric's)")
    ap.add_argument("--filters", type=int, default=None, help="override filter count")
    ap.add_argument("--topics", type=int, default=None,
                    help="topics per GPU per step (replicated, default 2M) / per batch (sharded, default: config's)")
    ap.add_argument("--mode", choices=["replicated", "sharded"], default=None,
                    help="replicated trie per GPU (default) or filter shards per GPU (default for --config 4)")
    ap.add_argument("--cpu-sample", type=int, default=1_500_000, help="topics timed on the host (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--check", type=int, default=20_000, help="topics checked bit-exactly vs the oracle")
    ap.add_argument("--streams", type=int, default=3,
                    help="streams the steps alternate over (batches overlap on the GPU; 1 = strictly serial)")
    ap.add_argument("--roof-steps", type=int, default=5,
                    help="serial steps after the timed region that time each kernel for the roofline")
    ap.add_argument("--walk", default=None, help="walk variant (queue|queue_xcd)")
    ap.add_argument("--ab", default=None, help="comma list of walk variants timed interleaved (extra report)")
    ap.add_argument("--stage-k", type=int, default=None)
    ap.add_argument("--lib", default=None, help="EXPERIMENT: alternative build of libtopicmatch.so (A/B of build options)")
    ap.add_argument("--hist", action="store_true", help="log per-level visit/probe histogram (diagnostic)")
    ap.add_argument("--presort", action="store_true",
                    help="EXPERIMENT: sort the batch by topic bytes on the host before upload (untimed)")
    ap.add_argument("--layout", type=int, default=None, help="1 = DFS relayout on commit (default), 0 = off")
    ap.add_argument("--presort-level", type=int, default=None,
                    help="EXPERIMENT: sort the batch by the word at this level on the host (untimed)")
    ap.add_argument("--opt", action="append", default=[], help="EXPERIMENT: engine option name=value (repeatable)")
    return ap.parse_args()


def main():
    a = parse()
    if a.lib:
        from emqx_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    rank, world, local = multi.env_rank()
    if world > 1:
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if (a.mode or ("sharded" if a.config == 4 else "replicated")) == "sharded":
        main_sharded(a, rank, world, local, dev)
        if world > 1:
            dist.destroy_process_group()
        return
    a.topics = a.topics or 2_000_000

    cfg = W.CONFIGS[a.config]
    n_filters = a.filters or cfg["filters"]
    t0 = time.time()
    fb, fo = W.filters(a.config, n=n_filters)
    log("rank %d: generated %d filters (%.1f MB) in %.1fs" % (rank, n_filters, fo[-1] / 1e6, time.time() - t0))
    t0 = time.time()
    eng = Engine(device=local, filters_hint=n_filters)
    if a.walk:
        eng.set_walk(a.walk)
    if a.stage_k:
        eng.set_option("stage_k", a.stage_k)
    if a.layout is not None:
        eng.set_option("layout", a.layout)
    for kv in a.opt:
        k, x = kv.split("=")
        eng.set_option(k, int(x))
    eng.insert_many(fb, fo)
    eng.commit()
    log("rank %d: trie built + committed in %.1fs: %d filters, %d nodes, image %.2f GB" % (
        rank, time.time() - t0, eng.filter_count, eng.node_count, eng.image_bytes / 1e9))

    tb, to = W.topics(a.config, n=a.topics, stream=multi.topic_stream(rank))
    n = len(to) - 1
    nbytes = int(to[-1])
    if a.presort or a.presort_level is not None:
        ts = [bytes(tb[to[i]:to[i + 1]]) for i in range(n)]
        if a.presort_level is not None:   # by the word at one level (then the whole topic)
            lv = a.presort_level
            ts.sort(key=lambda t: (t.split(b"/")[lv:lv + 1], t))
        else:
            ts.sort()
        lens = np.fromiter((len(t) for t in ts), dtype=np.uint64, count=n)
        to = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(lens, out=to[1:])
        tb = np.frombuffer(b"".join(ts), dtype=np.uint8).copy()
        del ts
        log("presorted %d topics (experiment, untimed)" % n)
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    d_c = torch.empty(n, dtype=torch.int32, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_t = torch.zeros(1, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)

    # size the output from one counting pass (untimed), with exact stats
    eng.set_stats(True)
    if a.hist:
        eng.set_option("hist", 1)
    eng.match_batch_device(d_b, d_o, n, nbytes, d_c, d_oo, None, 0, d_t, stream=st)
    torch.cuda.synchronize(dev)
    stats = eng.last_stats()
    if a.hist:
        import ctypes
        h = (ctypes.c_uint64 * 56)()
        eng.lib.tm_debug_hist(eng.h, h, 56)
        for k, name in enumerate(["visits", "probe_loads", "failed_probes"]):
            log("per-level %s per topic: %s" % (name, [round(h[16 * k + l] / n, 2) for l in range(16)]))
        log("visits reached by: inline literal %.2f, table literal %.2f, '+' %.2f per topic"
            % (h[48] / n, h[49] / n, h[50] / n))
    eng.set_stats(False)
    total = int(d_t.item())
    cap = total + 1024
    fan = np.sort(d_c.cpu().numpy().view(np.uint32))
    fanout = {"mean": float(fan.mean()), "p50": int(fan[len(fan) // 2]), "p90": int(fan[int(len(fan) * 0.9)]),
              "p99": int(fan[int(len(fan) * 0.99)]), "max": int(fan[-1])}
    log("fan-out per topic: %s" % fanout)
    d_i = torch.empty(cap, dtype=torch.int32, device=dev)

    # consecutive steps alternate over a.streams streams, each with its own
    # output buffers: a batch's tokenizer / copy-out overlap its neighbours'
    # walks (the engine rotates its per-batch workspace slots likewise)
    lanes = [(st, d_c, d_oo, d_i, d_t)]
    for _ in range(1, a.streams):
        lanes.append((torch.cuda.Stream(device=dev), torch.empty_like(d_c), torch.empty_like(d_oo),
                      torch.empty_like(d_i), torch.zeros_like(d_t)))
    eng.set_option("slots", min(4, max(2, a.streams)))
    k_step = [0]

    def step():
        s_, c_, oo_, i_, t_ = lanes[k_step[0] % len(lanes)]
        k_step[0] += 1
        eng.match_batch_device(d_b, d_o, n, nbytes, c_, oo_, i_, cap, t_, stream=s_)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)

    if a.ab:
        # interleaved A/B of walk variants on the same image and batch
        # (rounds x variants, one process: methodology rule 24)
        res = {v: [] for v in a.ab.split(",")}

        def configure(v):   # "walk[@option=value[@...]]"
            parts = v.split("@")
            eng.set_walk(parts[0])
            eng.set_option("walk_bpc", 0)
            for kv in parts[1:]:
                k, x = kv.split("=")
                eng.set_option(k, int(x))
        for _ in range(5):
            for v in res:
                configure(v)
                step()
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                for _ in range(3):
                    step()
                torch.cuda.synchronize(dev)
                res[v].append((time.perf_counter() - t1) / 3 * 1e3)
                assert int(d_t.item()) == total
        log("A/B ms/step (median, min): " + ", ".join(
            "%s %.2f/%.2f" % (v, sorted(x)[len(x) // 2], min(x)) for v, x in res.items()))
        configure(a.walk or "queue_xcd")

    # ---- timed region: K steps, kernel events recorded on the launch stream;
    # barrier + sync on both sides, max over ranks (emqx_amd/multi.py)
    dt = multi.timed_region(step, a.steps, lambda: torch.cuda.synchronize(dev))
    assert int(d_t.item()) == total, "match total changed between steps"
    # per-kernel durations for the roofline: with batches overlapping, a
    # kernel's event interval also holds its neighbours' work, so the kernels
    # are timed over a.roof_steps extra steps issued serially on one stream
    torch.cuda.synchronize(dev)
    eng.set_timing(True)
    for _ in range(a.roof_steps):
        eng.match_batch_device(d_b, d_o, n, nbytes, d_c, d_oo, d_i, cap, d_t, stream=st)
    torch.cuda.synchronize(dev)
    kms = eng.last_kernel_times()
    eng.set_timing(False)
    for _, c_, oo_, i_, t_ in lanes[1:]:   # overlapping batches: identical results in every lane
        assert int(t_.item()) == total and torch.equal(c_, d_c) and torch.equal(oo_, d_oo) and \
            torch.equal(i_[:total], d_i[:total]), "batches on different streams disagree"

    # ---- bit-exact spot check of this rank's batch against the oracle
    check_ok = None
    o1 = None
    cpu = None
    if rank == 0 and (a.check > 0 or (world == 1 and a.cpu_sample > 0)):
        from oracle import O1   # checker / CPU baseline only
        t0 = time.time()
        o1 = O1(n_filters)
        o1.insert_many(fb, fo)
        log("oracle O1 built in %.1fs (%d nodes)" % (time.time() - t0, o1.node_count))
        threads = a.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count())
        if a.check > 0:
            k = min(a.check, n)
            ksub = to[: k + 1]
            oc, oo, oi = o1.match_ids(tb, ksub, threads=threads)
            dc = d_c[:k].cpu().numpy().view(np.uint32)
            doo = d_oo[: k + 1].cpu().numpy().view(np.uint64)
            di = d_i[: int(doo[-1])].cpu().numpy().view(np.uint32)
            check_ok = bool(np.array_equal(dc, oc) and np.array_equal(doo, oo) and np.array_equal(di, oi))
            log("bit-exact check of %d topics vs O1: %s" % (k, check_ok))
        if world == 1 and a.cpu_sample > 0:
            k = min(a.cpu_sample, n)
            secs, m, e = o1.match_batch(tb, to[: k + 1], threads=threads)
            cpu = {"value": k / secs, "unit": "topics/s", "cores": threads, "kind": "port",
                   "sample": "%d topics of the same batch against the same %d-filter trie, C restatement "
                             "of emqx_trie (string-path ids, ETS-like tables), %d pthreads, %.1f s"
                             % (k, n_filters, threads, secs)}
            log("cpu baseline: %.0f topics/s on %d threads" % (k / secs, threads))

    if rank == 0:
        topics_per_s = n * a.steps * world / dt
        levels = stats["levels"]
        B = 8 * levels + 16 * stats["edge_reads"] + 4 * stats["matches"]   # SURVEY §8(d), per launch
        # dominant kernel = the longest stage (the walk); B is what one launch
        # of it processes
        kname = max(kms, key=kms.get) if kms else None
        walk_ms = kms.get(kname, 0.0) if kname else 0.0
        achieved = B / (walk_ms * 1e-3) / 1e9 if walk_ms > 0 else None
        # HBM traffic of the walk from the committed PMC passes of this same
        # workload (tools/pmc_passes.sh -> tools/traffic.py); null otherwise
        traffic = None
        tpath = os.path.join(ROOT, "profiles", "traffic_c%d.json" % a.config)
        if os.path.exists(tpath) and kname == "walk":
            tj = json.load(open(tpath))
            tc = tj.get("config") or {}
            if tc.get("filters") == n_filters and tc.get("topics_per_gpu_step") == n and tc.get("levels") == cfg["levels"]:
                traffic = tj["traffic_bytes_per_launch"] / (walk_ms * 1e-3) / 1e9
        out = {
            "metric": METRIC,
            "value": topics_per_s,
            "unit": "topics/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "C%d: %d distinct wildcard filters replicated per GPU, %d-level topics, "
                                   "%d topics per GPU per step, steps alternating over %d streams" % (
                                       a.config, n_filters, cfg["levels"], n, a.streams),
                       "filters": n_filters, "topics_per_gpu_step": n, "levels": cfg["levels"],
                       "parallelism": "replicated trie x %d, topic batches sharded by rank" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                         "traffic_source": ("FETCH_SIZE+WRITE_SIZE per launch, profiles/traffic_c%d.json, over this "
                                            "run's walk time" % a.config) if traffic else None,
                         "kernel": {"walk": "tm_walk_queue (balanced NFA walk, one 16 B node-half load per step)"
                                    }.get(kname, kname),
                         "kernel_ms": walk_ms,
                         "kernel_ms_source": "HIP events around each kernel on its stream, %d serial steps after "
                                             "the timed region" % a.roof_steps,
                         "algorithmic_bytes_per_launch": B,
                         "per_topic": {"n": levels / n, "E": stats["edge_reads"] / n, "M": stats["matches"] / n,
                                       "visits": stats["visits"] / n, "leaf_visits": stats["leaf_visits"] / n,
                                       "probe_loads": stats["probe_loads"] / n}},
            "cpu_baseline": cpu,
            "kernel_ms": kms,
            "filter_hits_per_s": stats["matches"] * a.steps * world / dt,
            "fanout": fanout,
            "parity_check": check_ok,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def main_sharded(a, rank, world, local, dev):
    """Config C4: the filter set partitioned over the ranks by
    literal-prefix (one shard per GPU).  Every rank holds the same topic batch,
    walks it against its own sub-trie with order keys, then the ranks
    exchange per-topic keyed lists (all-to-all, RCCL over xGMI) and each
    merges the lists of its topic slice into emqx_trie:match/1 order on its
    GPU.  One step = walk + exchange + merge of one batch; `value` = batch
    topics / max-over-ranks step time (strong scaling: the batch and filter
    set are fixed, N GPUs share them)."""
    from emqx_amd import shard
    S = world
    cfg = W.CONFIGS[a.config]
    n_filters = a.filters or cfg["filters"]
    t0 = time.time()
    fb, fo = W.filters(a.config, n=n_filters)
    log("rank %d: generated %d filters (%.1f MB) in %.1fs" % (rank, n_filters, fo[-1] / 1e6, time.time() - t0))
    t0 = time.time()
    eng = shard.ShardEngine(local, S, rank, filters_hint=n_filters // S + 1)
    eng.set_option("stage_k", a.stage_k or (512 if S == 1 else 128))   # per-shard fan-out is ~1/S
    eng.insert_many(fb, fo)
    eng.commit()
    log("rank %d: shard %d/%d built + committed in %.1fs: %d filters, %d nodes, image %.2f GB" % (
        rank, rank, S, time.time() - t0, eng.filter_count, eng.node_count, eng.image_bytes / 1e9))

    n_topics = a.topics if a.topics else cfg["topics"]
    tb, to = W.topics(a.config, n=n_topics, stream=0)     # the same batch on every shard
    n = len(to) - 1
    nbytes = int(to[-1])
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    d_c = torch.empty(n, dtype=torch.int32, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_t = torch.zeros(1, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream(dev)

    eng.set_stats(True)
    eng.match_keys_device(d_b, d_o, n, nbytes, d_c, d_oo, None, None, 0, d_t, stream=st)
    torch.cuda.synchronize(dev)
    stats = eng.last_stats()
    eng.set_stats(False)
    total = int(d_t.item())
    cap = total + 1024
    d_i = torch.empty(cap, dtype=torch.int32, device=dev)
    d_k = torch.empty(cap, dtype=torch.int64, device=dev)
    b = shard.slices(n, S)
    m = b[rank + 1] - b[rank]
    # merge output: sized after one exchange (the received total is exact)
    merged = {}

    def walk():
        eng.match_keys_device(d_b, d_o, n, nbytes, d_c, d_oo, d_i, d_k, cap, d_t, stream=st)

    def exchange():
        return shard.exchange(d_c, d_oo, d_i, d_k, n, S, rank)

    def merge(x):
        rc, base, rid, rk, mm = x
        if "cap" not in merged:
            merged["cap"] = max(int(rid.numel()), 1) + 1024
            merged["c"] = torch.empty(max(mm, 1), dtype=torch.int32, device=dev)
            merged["o"] = torch.empty(mm + 1, dtype=torch.int64, device=dev)
            merged["g"] = torch.empty(merged["cap"], dtype=torch.int32, device=dev)
            merged["t"] = torch.zeros(1, dtype=torch.int64, device=dev)
        eng.merge_device(mm, rc, base, rid, rk, merged["c"], merged["o"], merged["g"], merged["cap"], merged["t"],
                         stream=st)

    def step():
        walk()
        merge(exchange())

    for _ in range(max(a.warmup, 1)):
        step()
    torch.cuda.synchronize(dev)
    dt = multi.timed_region(step, a.steps, lambda: torch.cuda.synchronize(dev))
    assert int(d_t.item()) == total, "match total changed between steps"
    # per-kernel durations for the roofline: with batches overlapping, a
    # kernel's event interval also holds its neighbours' work, so the kernels
    # are timed over a.roof_steps extra steps issued serially on one stream
    torch.cuda.synchronize(dev)
    eng.set_timing(True)
    for _ in range(a.roof_steps):
        eng.match_batch_device(d_b, d_o, n, nbytes, d_c, d_oo, d_i, cap, d_t, stream=st)
    torch.cuda.synchronize(dev)
    kms = eng.last_kernel_times()
    eng.set_timing(False)
    mtotal = int(merged["t"].item())

    # phase breakdown (untimed extra loops): walk / exchange / merge
    def phase(fn, k=3):
        multi.timed_region(lambda: None, 1, lambda: torch.cuda.synchronize(dev))
        t1 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t1) / k * 1e3
    x = exchange()
    phases = {"walk_ms": phase(walk), "exchange_ms": phase(exchange), "merge_ms": phase(lambda: merge(x))}

    check_ok = None
    if rank == 0 and a.check > 0 and n_filters <= 20_000_000:
        from oracle import O1   # checker only
        threads = a.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count())
        o1 = O1(n_filters)
        o1.insert_many(fb, fo)
        k = min(a.check, m)
        oc, oo, oi = o1.match_ids(tb, to[: k + 1], threads=threads)
        g2i = shard.gid_to_index(shard.shard_of_batch(fb, fo, S), S)
        mo = merged["o"][: k + 1].cpu().numpy().view(np.uint64)
        mg = merged["g"][: int(mo[-1])].cpu().numpy().view(np.uint32).astype(np.int64)
        check_ok = bool(np.array_equal(mo, oo) and np.array_equal(g2i[mg], oi.astype(np.int64)))
        log("bit-exact check of %d topics (rank 0 slice) vs O1: %s" % (k, check_ok))

    levels = stats["levels"]
    B = 8 * levels + 16 * stats["edge_reads"] + 4 * stats["matches"]
    walk_ms = kms.get("walk", 0.0)
    achieved = B / (walk_ms * 1e-3) / 1e9 if walk_ms > 0 else None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": n * a.steps / dt,
            "unit": "topics/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "C%d: %d distinct wildcard filters sharded by literal-prefix over %d GPU(s), "
                                   "%d-level topics, one %d-topic batch per step" % (
                                       a.config, n_filters, S, cfg["levels"], n),
                       "filters": n_filters, "topics_per_step": n, "levels": cfg["levels"],
                       "parallelism": "filter shards x %d, all-to-all of keyed match lists (RCCL), device merge"
                                      % S},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": None,
                         "kernel": "tm_walk_queue<KEYS> on rank 0's shard", "kernel_ms": walk_ms,
                         "algorithmic_bytes_per_launch": B},
            "cpu_baseline": None,
            "kernel_ms": kms,
            "phases_ms_rank0": phases,
            "shard0": {"filters": eng.filter_count, "nodes": eng.node_count, "image_gb": eng.image_bytes / 1e9,
                       "ids_walked": total, "ids_merged": mtotal},
            "parity_check": check_ok,
        }
        print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
