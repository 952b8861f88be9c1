"""bench.py — topic matches/sec at 10M wildcard filters on MI355X.

One step = one publish batch (bytes + offsets already resident in HBM)
through the whole hot path of emqx_trie:match/1: device tokenizer
(emqx_topic:words/1), NFA walk, CSR emission of the ordered match lists.

Workload: 10M distinct wildcard filters (8 levels max,
p+ 0.20, p# 0.05, Zipf(1.0) words over 16/64/256/1024/4096x4), replicated on
every GPU.  Strong scaling (default; SURVEY §8(d) C3, BASELINE configs[2]
"publish batches sharded across 2/4/8 MI355X"): one 8M-topic batch per step
split 1/2/4/8 ways over the ranks (rank r walks slice r).  The weak-scaling
figure (every rank walks its own 1M-topic batch per step, SURVEY's "also
1M/GPU") is reported beside it under "weak"; `--scaling weak` makes it the
headline.  Steps rotate over `--batches` distinct batches (no batch is
replayed back to back, so L2 / MALL never hold the previous step's topics).
No collective on the data path.  `value` = topics matched per second over
all ranks (max-over-ranks step time).  Every rank checks its own lists
against the oracle; `parity_check` is the AND over ranks.

Extra legs at N = 1 (not `value`): the CPU baseline (O1 = C restatement of
emqx_trie, on all host threads and on one; O3 = the same algorithm over
interned ids), the host-buffer path tm_match_batch (PCIe both ways
included), and the micro-batcher driven by 16 producer threads with one
submit per publish (the NIF's path).

Run: python bench.py [--gpus N --steps K --warmup W]
     torchrun --nproc-per-node N bench.py --gpus N ...
     python bench.py --single-process --gpus N   (one process, one engine over N GPUs: tm_open_devices)
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd.engine import check_total  # noqa: E402
from emqx_amd import multi  # noqa: E402
from emqx_amd import workload as W  # noqa: E402

METRIC = "topic matches/sec (whole node) at 10M wildcard filters; % HBM roofline"
# micro-batcher leg: the NIF's configuration, among the best points of tools/bench_batcher.py (profiles/r02_b)
BATCHER = {"producers": 16, "deadline_us": 200, "max_topics": 262144, "lanes_per_replica": 4, "callback_threads": 8}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)   # ~5 s timed at C3 8M: long enough for a busy sampler
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=3, help="SURVEY §8(d) config (3 = the metric's)")
    ap.add_argument("--filters", type=int, default=None, help="override filter count")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong (default, SURVEY §8(d) C3 / BASELINE configs[2]): one batch per step split over "
                         "the ranks; weak: a batch of --topics per rank per step")
    ap.add_argument("--topics", type=int, default=None,
                    help="topics per batch (strong, default the config's: 8M at C3) or per GPU (weak, default "
                         "--weak-topics)")
    ap.add_argument("--weak-topics", type=int, default=1_000_000,
                    help="topics per GPU of the weak-scaling figure reported beside the strong one (0 = skip)")
    ap.add_argument("--check-rank", type=int, default=2_000,
                    help="topics of each batch every rank > 0 checks bit-exactly vs O3")
    ap.add_argument("--batches", type=int, default=2, help="distinct batches the steps rotate over")
    ap.add_argument("--mode", choices=["replicated", "sharded", "routed"], default=None,
                    help="replicated trie per GPU (default), filter shards per GPU with a list exchange (sharded), "
                         "or routed shards: topics exchanged to the shard owning their first --depth levels")
    ap.add_argument("--depth", type=int, default=2, help="routed mode: routing depth (levels of the key)")
    ap.add_argument("--self-rccl", action="store_true",
                    help="routed / sharded modes: a rank's own part of every exchange over RCCL too (at world 1 "
                         "the launch then runs the RCCL transfers the ranks of a multi-GPU node run)")
    ap.add_argument("--shards", type=int, default=None,
                    help="routed mode in one process (--single-process): shards on GPU 0 (a one-GPU rehearsal)")
    ap.add_argument("--single-process", action="store_true",
                    help="one process drives --gpus GPUs through ONE engine (tm_open_devices)")
    ap.add_argument("--replicas", default=None,
                    help="single-process: comma list of HIP ordinals (repeats allowed), default 0..gpus-1")
    ap.add_argument("--cpu-sample", type=int, default=1_500_000, help="topics timed on the host (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=None)
    ap.add_argument("--check", type=int, default=20_000, help="topics of each batch checked bit-exactly vs O1")
    ap.add_argument("--stream-kind", choices=["pool", "prio"], default="prio",
                    help="lane streams: high priority (default: a hardware queue each) or torch's pool (normal "
                         "priority: two of three lanes shared a queue, profiles/r05_u)")
    ap.add_argument("--streams", type=int, default=3,
                    help="streams the steps alternate over (batches overlap on the GPU; 1 = strictly serial)")
    ap.add_argument("--roof-steps", type=int, default=20,
                    help="serial steps after the timed region that time each kernel for the roofline")
    ap.add_argument("--no-extras", action="store_true", help="skip the host-buffer and batcher legs")
    ap.add_argument("--walk", default=None, help="walk variant (queue|queue_xcd)")
    ap.add_argument("--stage-k", type=int, default=None)
    ap.add_argument("--lib", default=None, help="EXPERIMENT: alternative build of libtopicmatch.so (A/B of build options)")
    ap.add_argument("--hist", action="store_true", help="log per-level visit/probe histogram (diagnostic)")
    ap.add_argument("--layout", type=int, default=None, help="1 = DFS relayout on commit (default), 0 = off")
    ap.add_argument("--opt", action="append", default=[], help="EXPERIMENT: engine option name=value (repeatable)")
    ap.add_argument("--presort", default=None, help="EXPERIMENT: batches sorted on the host: bytes | hN (N-bit word hashes)")
    ap.add_argument("--ab-opt", action="append", default=[],
                    help="EXPERIMENT: after the headline region, time the same batches again with these engine options "
                         "(name=value[,name=value]; repeatable; one trie build for every variant), reported under ab")
    return ap.parse_args()


def kernel_src_sha():
    """hash of the walk's sources (as tools/traffic.py records it with the PMC passes)"""
    import hashlib
    h = hashlib.sha256()
    for f in ("kernels.hip", "image.h", "kernels.h"):
        h.update(open(os.path.join(ROOT, "emqx_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:16]


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def host_cpus():
    """the CPUs this process may run on ("all host cores"):
    the scheduler affinity mask, plus the cgroup v2 CPU quota when one is set
    (quota / period CPUs), as evidence for the line"""
    aff = sorted(os.sched_getaffinity(0))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            quota = None if q == "max" else int(q) / int(per)
        except (OSError, ValueError):
            pass
    return {"affinity_cpus": len(aff), "affinity_first_last": [aff[0], aff[-1]] if aff else None,
            "cgroup_cpu_max_cpus": quota, "nproc": os.cpu_count()}


def host_threads(a):
    """threads of the all-cores CPU legs: every CPU of the affinity mask"""
    return a.cpu_threads or len(os.sched_getaffinity(0))


def insert_progress(eng, fb, fo, rank, chunk=10_000_000):
    """insert_many in slices of `chunk` filters with a log line per slice
    (a 100M-filter build takes minutes: the GPU job runner wants output)"""
    n = len(fo) - 1
    t0 = time.time()
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        eng.insert_many(fb[int(fo[lo]):int(fo[hi])], (fo[lo:hi + 1] - fo[lo]).astype(np.uint64))
        if n > chunk:
            log("rank %d: inserted %d / %d filters (%.0fs)" % (rank, hi, n, time.time() - t0))


def make_batches(a, cfg, rank, world):
    """this rank's topic batches: strong = slice `rank` of each global batch,
    weak = batches of its own stream"""
    out = []
    for b in range(a.batches):
        if a.scaling == "strong":
            tb, to = W.topics(a.config, n=a.topics, stream=b)
            lo, hi = multi.batch_slice(len(to) - 1, world, rank)
            sub = (to[lo:hi + 1] - to[lo]).astype(np.uint64)
            out.append((np.ascontiguousarray(tb[int(to[lo]):int(to[hi]) + 8]), sub))
        else:
            out.append(W.topics(a.config, n=a.topics, stream=multi.topic_stream(rank) * 64 + b))
    if a.presort:   # EXPERIMENT: the batch in topic byte order (lanes of a wave walk shared prefixes)
        from emqx_amd.engine import pack
        import zlib
        if a.presort == "lpt":   # the predicted-heavy topics first within each XCD range (tail experiment)
            import math

            def cost(t):   # hot words (low Zipf rank k of w<level>_<k>) lead to more filters below
                c = 0.0
                for w in t.split(b"/"):
                    k = w.rsplit(b"_", 1)[-1]
                    c += -math.log2(int(k) + 2) if k.isdigit() else -32
                return c
            res = []
            for tb, to in out:
                ts = W.unpack(tb, to)
                n = len(ts)
                srt = []
                for r in range(8):
                    srt += sorted(ts[n * r // 8: n * (r + 1) // 8], key=cost, reverse=True)
                res.append(pack(srt))
            return res
        if a.presort == "bytes":
            key = None
        else:   # "hN": each level's word hashed to N bits, level-major (what a device radix sort could use)
            nb = int(a.presort[1:])

            def key(t):
                return tuple(zlib.crc32(w) & ((1 << nb) - 1) for w in t.split(b"/"))
        out = [pack(sorted(W.unpack(tb, to), key=key)) for tb, to in out]
    return out


def median_leg(match, tb, to, k, th):
    """1 warm-up, then the median of 5 timed runs, each over its
    own fifth of the first k topics (k topics timed in all)"""
    k = max(5, k)
    match(tb, to[: k // 10 + 2], th)   # warm-up (caches, thread pool)
    rates = []
    for r in range(5):
        lo, hi = k * r // 5, k * (r + 1) // 5
        sub = (to[lo:hi + 1] - to[lo]).astype(np.uint64)
        secs = match(np.ascontiguousarray(tb[int(to[lo]):int(to[hi]) + 8]), sub, th)
        rates.append((hi - lo) / secs)
    rates.sort()
    return {"value": rates[2], "threads": th, "topics": k, "runs": [round(x) for x in rates],
            "method": "1 warm-up, median of 5 runs of %d topics" % (k // 5)}


def cpu_baseline(a, fb, fo, n_filters, tb, to):
    """O1 (the C restatement of emqx_trie: string-path ids, ETS-like tables)
    on all host threads and on one; O3 (interned ids) likewise"""
    from oracle import O1, O3   # checker / CPU baseline only
    threads = host_threads(a)
    n = len(to) - 1
    res = {}
    t0 = time.time()
    o3 = O3(n_filters)
    o3.insert_many(fb, fo)
    log("O3 built in %.1fs" % (time.time() - t0))
    legs = [("o3_all", min(a.cpu_sample, n), threads), ("o3_1core", min(a.cpu_sample // 8, n), 1)]
    for name, k, th in legs:
        res[name] = median_leg(lambda b, o, t: o3.match_batch(b, o, threads=t)[0], tb, to, k, th)
        log("cpu %s: %.0f topics/s (%d topics, %d threads)" % (name, res[name]["value"], k, th))
    o3.close()
    return res


def check_lists(oracle, a, k, batches, results):
    """the first k topics of each batch: device counts, offsets and ids
    equal the oracle's, id for id"""
    ok = True
    for (tb, to), (dc, doo, di) in zip(batches, results):
        kk = min(k, len(to) - 1)
        oc, oo, oi = oracle.match_ids(tb, to[: kk + 1], threads=host_threads(a))
        ok = ok and bool(np.array_equal(dc[:kk], oc) and np.array_equal(doo[: kk + 1], oo) and
                         np.array_equal(di[: int(oo[-1])], oi))
    return ok


def o3_check(a, fb, fo, n_filters, batches, results, k=None, extra=None):
    """filter sets too large for O1's string-path tables (C4: 100M filters),
    and the ranks > 0 of a multi-GPU run: the check runs against O3, the
    same algorithm over interned ids"""
    from oracle import O3   # checker only
    k = a.check if k is None else k
    t0 = time.time()
    o3 = O3(n_filters)
    o3.insert_many(fb, fo)
    log("oracle O3 built in %.1fs" % (time.time() - t0))
    ok = check_lists(o3, a, k, batches, results)
    if extra:
        ok = ok and check_lists(o3, a, k, *extra)
    log("bit-exact check of %d topics of each of %d batches vs O3: %s" % (min(k, len(batches[0][1]) - 1),
                                                                          len(batches) + (len(extra[0]) if extra
                                                                                          else 0), ok))
    o3.close()
    return ok


def o1_check_and_baseline(a, fb, fo, n_filters, batches, results, do_cpu, extra=None):
    from oracle import O1   # checker / CPU baseline only
    if n_filters > 20_000_000:
        return o3_check(a, fb, fo, n_filters, batches, results, extra=extra), {}
    t0 = time.time()
    o1 = O1(n_filters)
    o1.insert_many(fb, fo)
    log("oracle O1 built in %.1fs (%d nodes)" % (time.time() - t0, o1.node_count))
    threads = host_threads(a)
    ok = check_lists(o1, a, a.check, batches, results)
    if extra:
        ok = ok and check_lists(o1, a, a.check, *extra)
    log("bit-exact check of %d topics of each of %d batches vs O1: %s" % (min(a.check, len(batches[0][1]) - 1),
                                                                          len(batches) + (len(extra[0]) if extra
                                                                                          else 0), ok))
    legs = {}
    if do_cpu:
        tb, to = batches[0]
        n = len(to) - 1
        legs_o1 = [("o1_all", min(a.cpu_sample, n), threads)]
        if threads != 16:   # the 16-thread leg of round 2's lines, for continuity
            legs_o1.append(("o1_16", min(a.cpu_sample, n), 16))
        legs_o1.append(("o1_1core", min(a.cpu_sample // 30, n), 1))
        for name, k, th in legs_o1:
            legs[name] = median_leg(lambda b, o, t: o1.match_batch(b, o, threads=t)[0], tb, to, k, th)
            log("cpu %s: %.0f topics/s (%d topics, %d threads)" % (name, legs[name]["value"], k, th))
    o1.close()
    return ok, legs


def effective_cores(hc):
    """the CPUs' worth of time the CPU legs can use: the cgroup quota when one
    is set (the GPU box: 256 CPUs in the affinity mask, 16 CPUs of cpu.max),
    else the affinity count"""
    q = hc.get("cgroup_cpu_max_cpus")
    return max(1, int(round(q))) if q else hc["affinity_cpus"]


def cpu_line(a, legs, n_filters):
    th = host_threads(a)
    hc = host_cpus()
    return {"value": legs["o1_all"]["value"], "unit": "topics/s", "cores": effective_cores(hc), "kind": "port",
            "sample": "%d topics of the bench batch against the same %d-filter trie: O1, the C "
                      "restatement of emqx_trie (string-path node ids, ETS-like {trie_edge, NodeId, "
                      "Word} tables), %d pthreads over %d CPUs of the affinity mask sharing %s CPUs of cgroup "
                      "time, 1 warm-up then the median of 5 runs of %d topics"
                      % (legs["o1_all"]["topics"], n_filters, th, hc["affinity_cpus"],
                         hc["cgroup_cpu_max_cpus"] if hc["cgroup_cpu_max_cpus"] else "all",
                         legs["o1_all"]["topics"] // 5),
            "cores_source": "cgroup cpu.max quota" if hc["cgroup_cpu_max_cpus"] else "affinity mask",
            "affinity_cpus": hc["affinity_cpus"], "threads_used": th,
            "cpu_model": cpu_model(), "nproc": os.cpu_count(), "host_cpus": hc, "legs": legs}


# The one JSON line goes to the process's original stdout; everything else
# written to fd 1 -- RCCL's version banner at communicator init, library
# prints -- is sent to stderr, so stdout holds exactly the result line.
_RESULT_FD = None


def quiet_stdout():
    global _RESULT_FD
    if _RESULT_FD is None:
        sys.stdout.flush()
        _RESULT_FD = os.dup(1)
        os.dup2(2, 1)


def emit(obj):
    line = (json.dumps(obj) + "\n").encode()
    os.write(_RESULT_FD if _RESULT_FD is not None else 1, line)


def main():
    quiet_stdout()
    a = parse()
    if a.lib:
        from emqx_amd import _lib
        _lib.LIB_PATH = os.path.abspath(a.lib)
    rank, world, local = multi.env_rank()
    if a.single_process and a.mode == "routed":
        return main_routed_single(a)
    if a.single_process:
        return main_single_process(a)
    # TM_BENCH_SHARE_GPU=1 (rehearsal on a one-GPU box): every rank on GPU 0,
    # the control plane (barrier, max of step times) over gloo
    share = os.environ.get("TM_BENCH_SHARE_GPU") == "1"
    if share:
        local = 0
    if world > 1:
        dist.init_process_group("nccl" if torch.cuda.is_available() and not share else "gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # replicated whenever the trie fits one GPU's HBM (north_star): C4's 100M
    # filters (252M nodes) included; --mode sharded for filter sets beyond it
    if (a.mode or "replicated") == "sharded":
        main_sharded(a, rank, world, local, dev)
        if world > 1:
            dist.destroy_process_group()
        return
    if a.mode == "routed":
        main_routed(a, rank, world, local, dev)
        if world > 1:
            dist.destroy_process_group()
        return
    cfg = W.CONFIGS[a.config]
    # per step: the whole batch (strong) or each rank's (weak)
    a.topics = a.topics or (cfg["topics"] if a.scaling == "strong" else a.weak_topics)
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
    insert_progress(eng, fb, fo, rank)
    eng.commit()
    log("rank %d: trie built + committed in %.1fs: %d filters, %d nodes, image %.2f GB" % (
        rank, time.time() - t0, eng.filter_count, eng.node_count, eng.image_bytes / 1e9))
    eng.set_option("slots", min(4, max(2, a.streams)))

    # the headline region: strong = this rank's slice of each global batch,
    # weak = this rank's own batches (--scaling weak)
    t0 = time.time()
    batches = make_batches(a, cfg, rank, world)
    log("rank %d: %d batches of %d topics generated in %.1fs" % (rank, len(batches), len(batches[0][1]) - 1,
                                                                 time.time() - t0))
    # the lanes' streams, made once and shared by every region of the run:
    # a second set of high-priority streams (the weak leg's) shared the
    # process's few high-priority hardware queues with the first, and the
    # weak 1M step took 1.59 instead of 1.51 ms (profiles/r06_ab/ab_r04.jsonl)
    lane_streams = [Region.make_stream(dev, a.stream_kind) for _ in range(max(1, a.streams))]
    reg = Region(eng, dev, batches, lane_streams, stats=True, hist=a.hist)
    stats, fanout = reg.stats, reg.fanout
    log("fan-out per topic: %s" % fanout)
    reg.warm(a.warmup)
    # ---- timed region: K steps; barrier + sync on both sides, max over ranks
    dt = reg.timed(a.steps)
    kms = reg.kernel_times(a.roof_steps)
    xcd = reg.walk_clocks()
    if xcd:
        log("walk per XCD (ms): " + " | ".join("%d: %.3f %.3f %.3f %d" % (i, x["start"], x["home_done"], x["end"],
                                                                          x["stolen_chunks"]) for i, x in enumerate(xcd)))
    results = reg.results()
    n0 = reg.dbat[0][2]

    # in-process A/B of engine options over the same trie and batches
    ab = []
    for spec in a.ab_opt:
        kv = [x.split("=") for x in spec.split(",") if x]
        for k, x in kv:
            eng.set_option(k, int(x))
        reg.warm(a.warmup)
        adt = reg.timed(a.steps)
        akms = reg.kernel_times(a.roof_steps)
        axcd = reg.walk_clocks()
        ares = reg.results()
        same = all(np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1]) and np.array_equal(x[2], y[2])
                   for x, y in zip(ares, results))
        ab.append({"opts": spec, "ms_per_step": adt / a.steps * 1e3, "kernel_ms": akms, "walk_xcd_ms": axcd,
                   "value": (a.topics if a.scaling == "strong" else n0 * world) * a.steps / adt,
                   "lists_equal_headline": bool(same)})
        log("A/B %s: %.3f ms per step, kernels %s, lists equal: %s" % (spec, adt / a.steps * 1e3, akms, same))
    # the other scaling figure beside it (not `value`): weak scaling at
    # SURVEY §8(d)'s 1M topics per GPU when the headline is strong
    weak = None
    wres, wbatches = None, None
    if a.scaling == "strong" and a.weak_topics > 0:
        wbatches = [W.topics(a.config, n=a.weak_topics, stream=multi.topic_stream(rank) * 64 + b)
                    for b in range(a.batches)]
        wreg = Region(eng, dev, wbatches, lane_streams)
        wreg.warm(a.warmup)
        wdt = wreg.timed(a.steps)
        wres = wreg.results()
        weak = {"value": a.weak_topics * world * a.steps / wdt, "unit": "topics/s", "topics_per_gpu": a.weak_topics,
                "ms_per_step": wdt / a.steps * 1e3, "steps": a.steps,
                "scaling": "weak: each rank walks its own %d-topic batch per step" % a.weak_topics}
        log("weak scaling (%d topics per GPU): %.0f topics/s, %.3f ms per step" % (a.weak_topics, weak["value"],
                                                                                  weak["ms_per_step"]))
        wreg.free()
    reg.free()

    extras = {}
    if world == 1 and not a.no_extras:
        extras = host_legs(a, eng, batches[0], reg.totals[0])

    # parity on EVERY rank: rank 0 against O1 (a.check topics of each batch;
    # at N = 1 also the CPU baseline), every other rank against O3 (the same
    # algorithm over interned ids, a.check_rank topics); the line's
    # parity_check is the AND over ranks
    check_ok, cpu, check_desc = None, None, None
    do_cpu = world == 1 and a.cpu_sample > 0
    if a.check > 0 or do_cpu:
        if rank == 0:
            check_ok, legs = o1_check_and_baseline(a, fb, fo, n_filters, batches, results, do_cpu,
                                                   extra=(wbatches, wres) if wres else None)
            if legs:
                legs.update(cpu_baseline(a, fb, fo, n_filters, *batches[0]))
                cpu = cpu_line(a, legs, n_filters)
        else:
            check_ok = o3_check(a, fb, fo, n_filters, batches, results, k=a.check_rank,
                                extra=(wbatches, wres) if wres else None)
        if world > 1:
            check_ok = multi.all_true(check_ok)
        check_desc = ("rank 0: first %d topics of each batch vs O1%s; ranks 1..%d: first %d topics of each "
                      "batch vs O3; AND over ranks" % (a.check, " (O3 past 20M filters)" if n_filters > 20_000_000
                                                       else "", world - 1, a.check_rank)) if world > 1 else \
            "first %d topics of each batch vs O1%s" % (a.check, " (O3 past 20M filters)"
                                                        if n_filters > 20_000_000 else "")
        if wres:
            check_desc += ", the weak-scaling batches likewise"

    if rank == 0:
        topics_per_step = a.topics if a.scaling == "strong" else n0 * world
        topics_per_s = topics_per_step * a.steps / dt
        levels = stats["levels"]
        B = 8 * levels + 16 * stats["edge_reads"] + 4 * stats["matches"]   # SURVEY §8(d), per launch of batch 0
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
            same_kernel = tj.get("kernel_src_sha") == kernel_src_sha()
            if same_kernel and tc.get("filters") == n_filters and tc.get("topics_per_gpu_step") == n0 and \
                    tc.get("levels") == cfg["levels"]:
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
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": "C%d: %d distinct wildcard filters replicated per GPU, %d-level topics, "
                                   "%s, steps rotating over %d distinct batches and %d streams" % (
                                       a.config, n_filters, cfg["levels"],
                                       ("one %d-topic batch per step split over %d GPU(s)" % (a.topics, world))
                                       if a.scaling == "strong" else "%d topics per GPU per step" % a.topics,
                                       a.batches, a.streams),
                       "filters": n_filters, "topics_per_step": int(topics_per_step),
                       "topics_per_gpu_step": n0, "levels": cfg["levels"],
                       "parallelism": "replicated trie x %d, %s" % (
                           world, "topic batch split by rank" if a.scaling == "strong" else "a topic batch per rank")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": traffic,
                         "traffic_frac": (traffic / HBM_PEAK_GBS) if traffic else None,
                         "traffic_source": ("FETCH_SIZE+WRITE_SIZE per launch from the PMC passes of the same kernel "
                                            "sources (profiles/traffic_c%d.json, kernel_src_sha %s), over this run's "
                                            "walk time" % (a.config, kernel_src_sha())) if traffic else None,
                         "kernel": {"walk": "tm_walk_queue (balanced NFA walk, one 16 B node-half load per step)"
                                    }.get(kname, kname),
                         "kernel_ms": walk_ms,
                         "kernel_ms_source": "HIP events around each kernel on its stream, %d serial steps of "
                                             "batch 0 after the timed region" % a.roof_steps,
                         "algorithmic_bytes_per_launch": B,
                         "topics_per_launch": n0,
                         "per_topic": {"n": levels / n0, "E": stats["edge_reads"] / n0, "M": stats["matches"] / n0,
                                       "visits": stats["visits"] / n0, "leaf_visits": stats["leaf_visits"] / n0,
                                       "probe_loads": stats["probe_loads"] / n0,
                                       "prunable_visits": stats.get("prunable_visits", 0) / n0}},
            "cpu_baseline": cpu,
            "kernel_ms": kms,
            "walk_xcd_ms": xcd,
            "filter_hits_per_s": stats["matches"] / n0 * topics_per_s,
            "fanout": fanout,
            "parity_check": check_ok,
            "parity_scope": check_desc,
        }
        if weak:
            out["weak"] = weak
        if ab:
            out["ab"] = ab
        out.update(extras)
        emit(out)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


class Region:
    """HBM-resident topic batches stepped over `streams` lanes: consecutive
    steps alternate over the lanes (each with its own output buffers, so a
    batch's tokenizer / copy-out overlap its neighbours' walks; the engine
    rotates its per-batch workspace slots likewise) and rotate over the
    distinct batches.  Outputs are sized by one untimed counting pass per
    batch (exact stats of batch 0 when `stats`)."""

    def __init__(self, eng, dev, batches, streams, stats=False, hist=False):
        self.eng, self.dev = eng, dev
        self.st = streams[0]   # explicit (handle 0 would select the engine's own stream)
        self.dbat = []
        for tb, to in batches:
            n = len(to) - 1
            self.dbat.append((torch.from_numpy(tb).to(dev), torch.from_numpy(to.view(np.int64)).to(dev), n,
                              int(to[-1])))
        self.totals = []
        self.stats = None
        for i, (d_b, d_o, n, nb) in enumerate(self.dbat):
            c = torch.empty(n, dtype=torch.int32, device=dev)
            oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
            t = torch.zeros(1, dtype=torch.int64, device=dev)
            eng.set_stats(stats and i == 0)
            if stats and i == 0 and hist:
                eng.set_option("hist", 1)
            eng.match_batch_device(d_b, d_o, n, nb, c, oo, None, 0, t, stream=self.st)
            torch.cuda.synchronize(dev)
            if stats and i == 0:
                self.stats = eng.last_stats()
                fan = np.sort(c.cpu().numpy().view(np.uint32))
                self.fanout = {"mean": float(fan.mean()), "p50": int(fan[len(fan) // 2]),
                               "p90": int(fan[int(len(fan) * 0.9)]), "p99": int(fan[int(len(fan) * 0.99)]),
                               "max": int(fan[-1])}
                if hist:   # the stats batch's slot, before the next batch takes another
                    h = (ctypes.c_uint64 * 56)()
                    eng.lib.tm_debug_hist(eng.h, h, 56)
                    for k, name in enumerate(["visits", "probe_loads", "failed_probes"]):
                        log("per-level %s per topic: %s" % (name, [round(h[16 * k + lv] / n, 2) for lv in range(16)]))
                    eng.set_option("hist", 0)
            self.totals.append(int(t.item()))
        eng.set_stats(False)
        self.cap = max(self.totals) + 1024
        nmax = max(x[2] for x in self.dbat)
        self.lanes = []
        for s_ in streams:
            self.lanes.append((s_, torch.empty(nmax, dtype=torch.int32, device=dev),
                               torch.empty(nmax + 1, dtype=torch.int64, device=dev),
                               torch.empty(self.cap, dtype=torch.int32, device=dev),
                               torch.zeros(1, dtype=torch.int64, device=dev)))
        self.k = 0
        self.last = {}

    @staticmethod
    def make_stream(dev, kind):
        """a lane's stream.  Each stream is fed to one hardware queue (4 per
        process for normal priority, GPU_MAX_HW_QUEUES): two lanes on one
        queue run in submission order, so a batch's tokenizer waits behind
        another lane's copy-out; high-priority streams come from a queue set
        of their own (tools/stream_queues.py, profiles/r05_t)"""
        if kind == "prio":
            return torch.cuda.Stream(device=dev, priority=-1)
        return torch.cuda.Stream(device=dev)

    def step(self):
        j = self.k
        self.k += 1
        s_, c_, oo_, i_, t_ = self.lanes[j % len(self.lanes)]
        bi = j % len(self.dbat)
        d_b, d_o, n, nb = self.dbat[bi]
        self.eng.match_batch_device(d_b, d_o, n, nb, c_, oo_, i_, self.cap, t_, stream=s_)
        self.last[j % len(self.lanes)] = bi   # a lane's outputs hold its latest batch

    def sync(self):
        torch.cuda.synchronize(self.dev)

    def warm(self, steps):
        for _ in range(steps):
            self.step()
        self.sync()

    def timed(self, steps):
        """K steps bracketed by barrier + device sync on both sides; max over ranks"""
        dt = multi.timed_region(self.step, steps, self.sync)
        for li, bi in self.last.items():   # every lane's last result is complete and exact
            assert int(self.lanes[li][4].item()) == self.totals[bi], "match total changed between steps"
        return dt

    def kernel_times(self, steps):
        """per-kernel durations for the roofline: with batches overlapping, a
        kernel's event interval also holds its neighbours' work, so the
        kernels are timed over `steps` extra serial steps of batch 0 on one
        stream"""
        d_b, d_o, n0, nb0 = self.dbat[0]
        s0, c0, oo0, i0, t0_ = self.lanes[0]
        self.sync()
        self.eng.set_timing(True)
        for _ in range(steps):
            self.eng.match_batch_device(d_b, d_o, n0, nb0, c0, oo0, i0, self.cap, t0_, stream=s0)
        self.sync()
        kms = self.eng.last_kernel_times()
        self.eng.set_timing(False)
        return kms

    def walk_clocks(self):
        """per XCD of the last walk (batch 0 after kernel_times): ms from the
        walk's first wave start to the XCD's first start, to its home range's
        exhaustion (from then on its waves steal or drain) and to its last
        wave's end, and the chunks it stole (engine diagnostic)"""
        out = (ctypes.c_double * 32)()
        f = self.eng.lib.tm_debug_walk_clocks
        f.restype = ctypes.c_int
        if f(self.eng.h, out) != 0 or all(out[4 * x] < 0 for x in range(8)):
            return None   # (a build without the walk's clocks: TM_WALK_CLOCKS)
        return [{"start": round(out[4 * x], 4), "home_done": round(out[4 * x + 1], 4), "end": round(out[4 * x + 2], 4),
                 "stolen_chunks": int(out[4 * x + 3])} for x in range(8)]


    def results(self):
        """every batch's full result (host arrays: counts, offsets, ids)"""
        s0, c0, oo0, i0, t0_ = self.lanes[0]
        out = []
        for bi, (d_b, d_o, n, nb) in enumerate(self.dbat):
            self.eng.match_batch_device(d_b, d_o, n, nb, c0, oo0, i0, self.cap, t0_, stream=s0)
            self.sync()
            if check_total(t0_, self.cap, "batch %d" % bi) != self.totals[bi]:
                raise RuntimeError("batch %d: total changed between passes" % bi)
            out.append((c0[:n].cpu().numpy().view(np.uint32).copy(), oo0[: n + 1].cpu().numpy().view(np.uint64).copy(),
                        i0[: self.totals[bi]].cpu().numpy().view(np.uint32).copy()))
        return out

    def free(self):
        self.dbat, self.lanes = [], []
        torch.cuda.empty_cache()


def host_legs(a, eng, batch, total):
    """the product paths a broker takes (N = 1): host buffers through
    tm_match_batch (topics up and lists down over PCIe included), and the
    micro-batcher fed one publish at a time by 16 producer threads"""
    tb, to = batch
    n = len(to) - 1
    out = {}
    # the caller stages topics and receives counts / offsets in pinned host
    # memory (as the batcher's lanes do); the ids come back into the
    # library's pinned output pool (tm_match_batch_owned)
    ptb = torch.from_numpy(tb).pin_memory().numpy()
    pto = torch.from_numpy(to.view(np.int64)).pin_memory().numpy().view(np.uint64)
    pc = torch.empty(n, dtype=torch.int32).pin_memory().numpy().view(np.uint32)
    po = torch.empty(n + 1, dtype=torch.int64).pin_memory().numpy().view(np.uint64)
    counts, offs, ids = eng.match_batch(ptb, pto, counts=pc, offs=po, keep=True)   # warm the workspace
    del ids
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        counts, offs, ids = eng.match_batch(ptb, pto, counts=pc, offs=po, keep=True)
        del ids
    secs = (time.perf_counter() - t0) / reps
    assert int(offs[-1]) == total
    moved = int(to[-1]) + 8 * (n + 1) + 4 * n + 8 * (n + 1) + 4 * total
    out["host_path"] = {"topics_per_s": n / secs, "ms_per_batch": secs * 1e3, "topics": n,
                        "pcie_bytes": moved, "pcie_gbs": moved / secs / 1e9,
                        "path": "tm_match_batch_owned (1M-topic chunks pipelined on two streams): pinned host topics -> HBM -> walk -> counts, offsets and ids "
                                "back to pinned host memory (one library-sized read-back), PCIe both ways included"}
    log("host path: %.0f topics/s, %.2f ms per %d-topic batch, %.1f GB/s over PCIe" % (
        n / secs, secs * 1e3, n, moved / secs / 1e9))
    lib_path = os.path.join(ROOT, "tools", "ubench", "libbatchdrive.so")
    if os.path.exists(lib_path):
        drv = ctypes.CDLL(lib_path)
        drv.tm_bench_batcher.restype = ctypes.c_int
        drv.tm_bench_batcher.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double)]
        k = n   # the whole batch, after a warm-up run inside the driver
        res = (ctypes.c_double * 14)()
        bc = BATCHER
        rc = drv.tm_bench_batcher(eng.h, tb.ctypes.data, to.ctypes.data, k, bc["producers"], bc["deadline_us"],
                                  bc["max_topics"], bc["lanes_per_replica"], 0, bc["callback_threads"], res)
        if rc == 0:
            out["batcher"] = dict(bc, topics_per_s=res[1], topics=k, batches=int(res[2]), mean_batch=res[3],
                                  lat_us_p50=res[4], lat_us_p99=res[5], failed=int(res[6]), matches=int(res[7]),
                                  per_batch_us={"sealed_to_lane": res[8], "pack": res[9], "device": res[10],
                                                "callbacks": res[11], "device_launch": res[12],
                                                "device_wait": res[13]},
                                  path="tm_batcher_submit per publish from %d threads, per-topic callbacks "
                                       "(NIF path), PCIe both ways included" % bc["producers"])
            log("batcher: %.0f topics/s, mean batch %.0f, p50 %.0f us, p99 %.0f us" % (res[1], res[3], res[4],
                                                                                     res[5]))
    return out


def main_single_process(a):
    """one process, one engine over N replicas (tm_open_devices): a
    resident batch slice on each replica's GPU, every step issues all N
    batches (device API, each on its GPU's stream) and waits for all — the
    whole node driven through the C-ABI the NIF uses"""
    devs = [int(x) for x in a.replicas.split(",")] if a.replicas else list(range(a.gpus))
    N = len(devs)
    cfg = W.CONFIGS[a.config]
    a.topics = a.topics or cfg["topics"]
    n_filters = a.filters or cfg["filters"]
    fb, fo = W.filters(a.config, n=n_filters)
    t0 = time.time()
    eng = Engine(devices=devs, filters_hint=n_filters)
    eng.insert_many(fb, fo)
    eng.commit()
    log("engine over %s built in %.1fs" % (devs, time.time() - t0))
    tb, to = W.topics(a.config, n=a.topics, stream=0)
    parts = []
    for r, d in enumerate(devs):
        dev = torch.device("cuda", d)
        lo, hi = multi.batch_slice(len(to) - 1, N, r)
        sub = (to[lo:hi + 1] - to[lo]).astype(np.uint64)
        sb = np.ascontiguousarray(tb[int(to[lo]):int(to[hi]) + 8])
        n = hi - lo
        with torch.cuda.device(dev):
            s_ = torch.cuda.Stream(device=dev)
        parts.append(dict(dev=dev, s=s_, b=torch.from_numpy(sb).to(dev), o=torch.from_numpy(sub.view(np.int64)).to(dev),
                          n=n, nb=int(sub[-1]), c=torch.empty(n, dtype=torch.int32, device=dev),
                          oo=torch.empty(n + 1, dtype=torch.int64, device=dev),
                          t=torch.zeros(1, dtype=torch.int64, device=dev)))
    for p in parts:   # exact output sizes
        eng.match_batch_device(p["b"], p["o"], p["n"], p["nb"], p["c"], p["oo"], None, 0, p["t"], stream=p["s"])
    for p in parts:
        torch.cuda.synchronize(p["dev"])
        p["cap"] = int(p["t"].item()) + 1024
        p["i"] = torch.empty(p["cap"], dtype=torch.int32, device=p["dev"])

    def step():
        for p in parts:
            eng.match_batch_device(p["b"], p["o"], p["n"], p["nb"], p["c"], p["oo"], p["i"], p["cap"], p["t"],
                                   stream=p["s"])

    def sync():
        for p in parts:
            torch.cuda.synchronize(p["dev"])
    for _ in range(a.warmup):
        step()
    dt = multi.timed_region(step, a.steps, sync)
    counts, offs, ids = eng.match_batch(tb, to)   # the host path over all replicas: the same lists
    got = np.concatenate([p["i"][: int(p["t"].item())].cpu().numpy().view(np.uint32) for p in parts])
    assert np.array_equal(got, ids), "replica results differ from the whole-batch host path"
    emit({"metric": METRIC, "value": a.topics * a.steps / dt, "unit": "topics/s", "n_gpus": N,
                      "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3,
                      "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32",
                      "data": "synthetic",
                      "config": {"workload": "C%d single process, one engine over replicas %s, one %d-topic batch "
                                             "per step split over them" % (a.config, devs, a.topics),
                                 "filters": n_filters, "topics_per_step": a.topics,
                                 "parallelism": "one process, tm_open_devices x %d" % N},
                      "replicas_consistent": True})
    eng.close()


def routed_line(a, cfg, n_filters, S, topics_per_step, dt, kms, stats, n0, eng_info, check_ok, phases, transport):
    levels = stats["levels"]
    B = 8 * levels + 16 * stats["edge_reads"] + 4 * stats["matches"]   # rank 0's owned batch, one launch
    walk_ms = kms.get("walk", 0.0)
    achieved = B / (walk_ms * 1e-3) / 1e9 if walk_ms > 0 else None
    return {
        "metric": METRIC, "value": topics_per_step * a.steps / dt, "unit": "topics/s", "n_gpus": S,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32", "data": "synthetic",
        "config": {"workload": "C%d: %d distinct wildcard filters routed over %d shard(s) by their first %d levels "
                               "(wildcard-led ones on every shard), %d-level topics, one %d-topic batch per step "
                               "split over the ranks; each topic walked on its owner shard only" % (
                                   a.config, n_filters, S, a.depth, cfg["levels"], topics_per_step),
                   "filters": n_filters, "topics_per_step": topics_per_step, "levels": cfg["levels"],
                   "depth": a.depth,
                   "parallelism": "routed shards x %d: topic all-to-all to the owner (%s), walk, lists back" % (
                       S, transport)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": None,
                     "kernel": "tm_walk_queue on rank 0's owned topics", "kernel_ms": walk_ms,
                     "algorithmic_bytes_per_launch": B, "topics_per_launch": n0},
        "cpu_baseline": None, "kernel_ms": kms, "phases_ms_rank0": phases, "shard0": eng_info,
        "parity_check": check_ok,
    }


def routed_check(a, fb, fo, n_filters, batches, results, rank):
    """every rank: its own batches' lists (returned to it, in its topic
    order) against O1 over the WHOLE filter set (O3 past 20M filters)"""
    from oracle import O1, O3   # checker only
    o = (O1 if n_filters <= 20_000_000 else O3)(n_filters)
    o.insert_many(fb, fo)
    k = a.check if rank == 0 else a.check_rank
    ok = check_lists(o, a, k, batches, results)
    o.close()
    log("rank %d: bit-exact check of %d topics of each batch vs %s over all filters: %s" % (
        rank, k, "O1" if n_filters <= 20_000_000 else "O3", ok))
    return ok


def main_routed(a, rank, world, local, dev):
    """Routed sharded mode, one process per GPU (RCCL): each rank holds the
    filters routed to it plus the wildcard-led ones (global ids), walks only
    the topics it owns, and returns their lists to the ranks that sent them."""
    from emqx_amd import shard
    S = world
    cfg = W.CONFIGS[a.config]
    n_filters = a.filters or cfg["filters"]
    a.topics = a.topics or cfg["topics"]
    fb, fo = W.filters(a.config, n=n_filters)
    t0 = time.time()
    eng = shard.RoutedEngine(local, S, rank, depth=a.depth, filters_hint=n_filters)
    eng.insert_many(fb, fo)
    eng.commit()
    info = {"filters": eng.filter_count, "nodes": eng.node_count, "image_gb": eng.image_bytes / 1e9,
            "filter_share": eng.filter_count / n_filters}
    log("rank %d: routed shard built in %.1fs: %s" % (rank, time.time() - t0, info))
    uid = [shard.Comm.unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0)
    comm = shard.Comm.init_rank(uid[0], S, rank, local)
    if a.self_rccl:
        comm.set_self_rccl(True)
    batches = make_batches(a, cfg, rank, world)   # strong: slice `rank` of each global batch
    st = torch.cuda.Stream(device=dev)
    dbat = []
    for tb, to in batches:
        pad = np.zeros(len(tb) + 16, dtype=np.uint8)
        pad[:len(tb)] = tb
        dbat.append((torch.from_numpy(pad).to(dev), torch.from_numpy(to.view(np.int64)).to(dev), len(to) - 1,
                     int(to[-1])))
    caps, mmax = [], 1
    for d_b, d_o, n, nb in dbat:   # sizes of the owned batches' lists (untimed)
        o = shard.route_exchange(comm, shard.route_in(n, nb, d_b, d_o, a.depth, st))
        c = torch.empty(max(o.m, 1), dtype=torch.int32, device=dev)
        oo = torch.empty(o.m + 1, dtype=torch.int64, device=dev)
        t = torch.zeros(1, dtype=torch.int64, device=dev)
        eng.match_batch_device(o.d_bytes, o.d_off, o.m, o.bytes, c, oo, None, 0, t, stream=st)
        torch.cuda.synchronize(dev)
        caps.append(int(t.item()) + 1024)
        mmax = max(mmax, o.m)
    cap = max(caps)
    d_c = torch.empty(mmax + 1, dtype=torch.int32, device=dev)
    d_oo = torch.empty(mmax + 2, dtype=torch.int64, device=dev)
    d_i = torch.empty(cap, dtype=torch.int32, device=dev)
    d_t = torch.zeros(1, dtype=torch.int64, device=dev)
    k_step = [0]
    last = {}

    def exchange(bi):
        d_b, d_o, n, nb = dbat[bi]
        return shard.route_exchange(comm, shard.route_in(n, nb, d_b, d_o, a.depth, st))

    def walk(o):
        eng.match_batch_device(o.d_bytes, o.d_off, o.m, o.bytes, d_c, d_oo, d_i, cap, d_t, stream=st)

    def back():
        return shard.route_return(comm, d_c, d_oo, d_i, stream=st)

    def step():
        bi = k_step[0] % len(dbat)
        k_step[0] += 1
        o = exchange(bi)
        walk(o)
        last["res"] = back()
        last["bi"] = bi

    for _ in range(max(a.warmup, 1)):
        step()
    torch.cuda.synchronize(dev)
    dt = multi.timed_region(step, a.steps, lambda: torch.cuda.synchronize(dev))
    # stats and kernel times of rank 0's owned batch 0 (serial, untimed)
    o = exchange(0)
    eng.set_stats(True)
    walk(o)
    torch.cuda.synchronize(dev)
    stats = eng.last_stats()
    eng.set_stats(False)
    n0 = o.m
    eng.set_timing(True)
    for _ in range(a.roof_steps):
        walk(o)
    torch.cuda.synchronize(dev)
    kms = eng.last_kernel_times()
    eng.set_timing(False)
    back()
    torch.cuda.synchronize(dev)

    def phase(fn, k=3):
        multi.timed_region(lambda: None, 1, lambda: torch.cuda.synchronize(dev))
        t1 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t1) / k * 1e3
    oo_ = exchange(0)
    phases = {"exchange_ms": phase(lambda: exchange(0)), "walk_ms": phase(lambda: walk(oo_)),
              "return_ms": phase(back)}
    # every batch's lists on this rank, in its topic order
    results = []
    for bi in range(len(dbat)):
        walk(exchange(bi))
        torch.cuda.synchronize(dev)
        check_total(d_t, cap, "routed owned batch %d" % bi)
        r = back()
        torch.cuda.synchronize(dev)
        results.append((shard._dev_array(r.d_counts, r.n, np.uint32, local),
                        shard._dev_array(r.d_offs, r.n + 1, np.uint64, local),
                        shard._dev_array(r.d_ids, r.total, np.uint32, local)))
    check_ok = None
    if a.check > 0:
        check_ok = routed_check(a, fb, fo, n_filters, batches, results, rank)
        if world > 1:
            check_ok = multi.all_true(check_ok)
    if rank == 0:
        emit(routed_line(a, cfg, n_filters, S, a.topics, dt, kms, stats, n0, info, check_ok, phases,
                         ("RCCL (own buckets too)" if a.self_rccl else "RCCL") if comm.rccl else "device copies"))
    comm.close()
    eng.close()


def main_routed_single(a):
    """Routed mode in ONE process: --shards S shard engines (on GPU 0 by
    default, or on --replicas) exchanging by device copies / RCCL group calls
    (tm_route_exchange_group): the launch rehearsal of the routed mode on a
    one-GPU box.  One step = every shard's slice of the batch routed, each
    shard's owned topics walked, the lists returned."""
    from emqx_amd import shard
    devs = [int(x) for x in a.replicas.split(",")] if a.replicas else [0] * (a.shards or a.gpus)
    S = len(devs)
    cfg = W.CONFIGS[a.config]
    n_filters = a.filters or cfg["filters"]
    a.topics = a.topics or cfg["topics"]
    fb, fo = W.filters(a.config, n=n_filters)
    t0 = time.time()
    rs = shard.RoutedSet(devs, depth=a.depth, filters_hint=n_filters)
    rs.insert_many(fb, fo)
    info = [{"filters": e.filter_count, "nodes": e.node_count, "image_gb": round(e.image_bytes / 1e9, 3),
             "filter_share": round(e.filter_count / n_filters, 4)} for e in rs.engines]
    log("%d routed shards built in %.1fs: %s" % (S, time.time() - t0, info))
    per_rank = [make_batches(a, cfg, r, S) for r in range(S)]   # [rank][batch]
    batches = [[per_rank[r][b] for r in range(S)] for b in range(a.batches)]
    # one step through RoutedSet's machinery, with HBM-resident inputs
    import ctypes as C
    from emqx_amd import _lib as L
    lib = rs.comms[0].lib
    hs = (C.c_void_p * S)(*[c.h.value for c in rs.comms])
    streams = [torch.cuda.Stream(device=torch.device("cuda", d)) for d in devs]
    dins = []
    for b in range(a.batches):
        ins = []
        keep = []
        for r, (tb, to) in enumerate(batches[b]):
            dev = torch.device("cuda", devs[r])
            pad = np.zeros(len(tb) + 16, dtype=np.uint8)
            pad[:len(tb)] = tb
            d_b, d_o = torch.from_numpy(pad).to(dev), torch.from_numpy(to.view(np.int64)).to(dev)
            keep.append((d_b, d_o))
            ins.append(shard.route_in(len(to) - 1, int(to[-1]), d_b, d_o, a.depth, streams[r]))
        dins.append(((L.TmRouteIn * S)(*ins), keep))
    state = {}

    def exchange(b):
        outs = (L.TmRouteOut * S)()
        rc = lib.tm_route_exchange_group(hs, S, dins[b][0], outs)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_route_exchange_group")
        return outs

    def lists_for(outs, sized=True):
        ls = []
        for r, e in enumerate(rs.engines):
            o = outs[r]
            buf = state.setdefault(r, {})
            dev = torch.device("cuda", devs[r])
            if buf.get("m", -1) < o.m:
                buf["m"] = o.m + 1024
                buf["c"] = torch.empty(buf["m"], dtype=torch.int32, device=dev)
                buf["o"] = torch.empty(buf["m"] + 1, dtype=torch.int64, device=dev)
                buf["t"] = torch.zeros(1, dtype=torch.int64, device=dev)
            if not sized or "cap" not in buf:
                e.match_batch_device(o.d_bytes, o.d_off, o.m, o.bytes, buf["c"], buf["o"], None, 0, buf["t"],
                                     stream=streams[r])
                streams[r].synchronize()
                need = int(buf["t"].item()) + 1024
                if buf.get("cap", 0) < need:
                    buf["cap"] = need * 2
                    buf["i"] = torch.empty(buf["cap"], dtype=torch.int32, device=dev)
            e.match_batch_device(o.d_bytes, o.d_off, o.m, o.bytes, buf["c"], buf["o"], buf["i"], buf["cap"],
                                 buf["t"], stream=streams[r])
            ls.append(L.TmRouteLists(buf["c"].data_ptr(), buf["o"].data_ptr(), buf["i"].data_ptr(),
                                     streams[r].cuda_stream))
        return (L.TmRouteLists * S)(*ls)

    def back(ls):
        res = (L.TmRouteResult * S)()
        rc = lib.tm_route_return_group(hs, S, ls, res)
        if rc != L.TM_OK:
            raise L.TopicMatchError(rc, "tm_route_return_group")
        return res

    for b in range(a.batches):   # size every shard's output for every batch (untimed)
        back(lists_for(exchange(b), sized=False))
    k_step = [0]

    def step():
        b = k_step[0] % a.batches
        k_step[0] += 1
        state["res"] = back(lists_for(exchange(b)))

    def sync():
        for d in sorted(set(devs)):
            torch.cuda.synchronize(torch.device("cuda", d))
    for _ in range(max(a.warmup, 1)):
        step()
    sync()
    dt = multi.timed_region(step, a.steps, sync)
    # rank 0's owned batch 0: stats and kernel times
    outs = exchange(0)
    ls = lists_for(outs)
    sync()
    e0, o0 = rs.engines[0], outs[0]
    buf = state[0]
    e0.set_stats(True)
    e0.match_batch_device(o0.d_bytes, o0.d_off, o0.m, o0.bytes, buf["c"], buf["o"], buf["i"], buf["cap"], buf["t"],
                          stream=streams[0])
    sync()
    stats = e0.last_stats()
    e0.set_stats(False)
    e0.set_timing(True)
    for _ in range(a.roof_steps):
        e0.match_batch_device(o0.d_bytes, o0.d_off, o0.m, o0.bytes, buf["c"], buf["o"], buf["i"], buf["cap"],
                              buf["t"], stream=streams[0])
    sync()
    kms = e0.last_kernel_times()
    e0.set_timing(False)
    back(ls)
    sync()
    check_ok = True
    for b in range(a.batches):
        res = back(lists_for(exchange(b)))
        sync()
        for r in range(S):
            x = res[r]
            got = (shard._dev_array(x.d_counts, x.n, np.uint32, devs[r]),
                   shard._dev_array(x.d_offs, x.n + 1, np.uint64, devs[r]),
                   shard._dev_array(x.d_ids, x.total, np.uint32, devs[r]))
            state.setdefault("results", {})[(r, b)] = got
    if a.check > 0:
        from oracle import O1, O3   # checker only
        o = (O1 if n_filters <= 20_000_000 else O3)(n_filters)
        o.insert_many(fb, fo)
        for (r, b), got in state["results"].items():
            check_ok = check_ok and check_lists(o, a, a.check_rank if r else a.check, [batches[b][r]], [got])
        o.close()
        log("bit-exact check of every shard's batches vs the whole filter set: %s" % check_ok)
    line = routed_line(a, cfg, n_filters, S, a.topics, dt, kms, stats, o0.m, info[0], check_ok if a.check else None,
                       None, "device copies" if not rs.comms[0].rccl else "RCCL group")
    line["n_gpus"] = len(set(devs))
    line["config"]["parallelism"] += ", one process, shards on GPUs %s" % devs
    line["shards"] = info
    emit(line)
    rs.close()


def main_sharded(a, rank, world, local, dev):
    """Config C4: the filter set partitioned over the ranks by
    literal prefix (one shard per GPU).  Every rank holds the same topic batch,
    walks it against its own sub-trie with order keys, then the ranks
    exchange per-topic keyed lists natively over RCCL (tm_shard_exchange: an
    all-to-all, each id crosses xGMI once) and each merges the lists of its
    topic slice into emqx_trie:match/1 order on its GPU.  One step = walk +
    exchange + merge of one batch; `value` = batch topics / max-over-ranks
    step time (strong scaling: the batch and filter set are fixed, N GPUs
    share them)."""
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
    # one RCCL communicator over the ranks, its id shared over torch.distributed
    uid = [shard.Comm.unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(uid, src=0)
    comm = shard.Comm.init_rank(uid[0], S, rank, local)
    if a.self_rccl:
        comm.set_self_rccl(True)

    n_topics = a.topics if a.topics else cfg["topics"]
    tb, to = W.topics(a.config, n=n_topics, stream=0)     # the same batch on every shard
    n = len(to) - 1
    nbytes = int(to[-1])
    KW = shard.key_words_for(tb, to)
    d_b = torch.from_numpy(tb).to(dev)
    d_o = torch.from_numpy(to.view(np.int64)).to(dev)
    d_c = torch.empty(n, dtype=torch.int32, device=dev)
    d_oo = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d_t = torch.zeros(1, dtype=torch.int64, device=dev)
    # one explicit stream orders walk -> RCCL exchange -> merge (the legacy
    # default stream's handle 0 would select the engine's / comm's own)
    st = torch.cuda.Stream(device=dev)

    eng.set_stats(True)
    eng.match_keys_device(d_b, d_o, n, nbytes, d_c, d_oo, None, None, 0, d_t, stream=st, key_words=KW)
    torch.cuda.synchronize(dev)
    stats = eng.last_stats()
    eng.set_stats(False)
    total = int(d_t.item())
    cap = total + 1024
    d_i = torch.empty(cap, dtype=torch.int32, device=dev)
    d_k = torch.empty(cap * KW, dtype=torch.int64, device=dev)
    b = shard.slices(n, S)
    m = b[rank + 1] - b[rank]
    merged = {}

    def walk():
        eng.match_keys_device(d_b, d_o, n, nbytes, d_c, d_oo, d_i, d_k, cap, d_t, stream=st, key_words=KW)

    def exchange():
        return shard.exchange_native(comm, d_c, d_oo, d_i, d_k, n, key_words=KW, key_stride=cap, stream=st)

    def merge(x):
        if merged.get("cap", 0) < x.total + 1:
            merged["cap"] = x.total + 1 + 1024
            merged["c"] = torch.empty(max(x.m, 1), dtype=torch.int32, device=dev)
            merged["o"] = torch.empty(x.m + 1, dtype=torch.int64, device=dev)
            merged["g"] = torch.empty(merged["cap"], dtype=torch.int32, device=dev)
            merged["t"] = torch.zeros(1, dtype=torch.int64, device=dev)
        eng.merge_device(x.m, x.d_counts, x.d_src_base, x.d_ids, x.d_keys, merged["c"], merged["o"], merged["g"],
                         merged["cap"], merged["t"], stream=st, key_words=KW, key_stride=x.total)

    def step():
        walk()
        merge(exchange())

    for _ in range(max(a.warmup, 1)):
        step()
    torch.cuda.synchronize(dev)
    dt = multi.timed_region(step, a.steps, lambda: torch.cuda.synchronize(dev))
    assert int(d_t.item()) == total, "match total changed between steps"
    # the dominant kernel of this mode is the KEYED walk: time it serially
    torch.cuda.synchronize(dev)
    eng.set_timing(True)
    for _ in range(a.roof_steps):
        walk()
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
        o1 = O1(n_filters)
        o1.insert_many(fb, fo)
        k = min(a.check, m)
        oc, oo, oi = o1.match_ids(tb, to[: k + 1], threads=host_threads(a))
        g2i = shard.gid_to_index(shard.shard_of_batch(fb, fo, S), S)
        mo = merged["o"][: k + 1].cpu().numpy().view(np.uint64)
        mg = merged["g"][: int(mo[-1])].cpu().numpy().view(np.uint32).astype(np.int64)
        check_ok = bool(np.array_equal(mo, oo) and np.array_equal(g2i[mg], oi.astype(np.int64)))
        log("bit-exact check of %d topics (rank 0 slice) vs O1: %s" % (k, check_ok))

    levels = stats["levels"]
    B = 8 * levels + 16 * stats["edge_reads"] + 4 * stats["matches"] + 8 * stats["matches"] * KW   # + the keys
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
                       "parallelism": "filter shards x %d, RCCL all-to-all of keyed match lists "
                                      "(tm_shard_exchange, %s), device merge" % (
                                          S, "RCCL" if comm.rccl else "device copies")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": None,
                         "kernel": "tm_walk_queue<KEYS> (keyed walk) on rank 0's shard", "kernel_ms": walk_ms,
                         "algorithmic_bytes_per_launch": B},
            "cpu_baseline": None,
            "kernel_ms": kms,
            "phases_ms_rank0": phases,
            "shard0": {"filters": eng.filter_count, "nodes": eng.node_count, "image_gb": eng.image_bytes / 1e9,
                       "ids_walked": total, "ids_merged": mtotal},
            "parity_check": check_ok,
        }
        emit(out)
    comm.close()
    eng.close()


if __name__ == "__main__":
    main()
