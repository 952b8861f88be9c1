"""Driver of the walk cache model (tools/sim/walksim.cpp; diagnostic only).

Builds a host-only engine (device = -1: the host mirror and its relayout,
no GPU) over a config's filters, exports the laid-out image and one XCD's
share of a batch's tokenized topics, and replays the walk through the cache
model for each requested layout.  Prints one JSON line per layout with
per-topic loads, L1->L2 requests and L2 misses (the fabric read requests the
PMC pass counts as TCC_EA0_RDREQ) by kind.

  python tools/sim/run_sim.py --config 3 --topics 1000000 --layouts cur,slotrec+occ5,pair
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from emqx_amd import Engine  # noqa: E402
from emqx_amd import workload as W  # noqa: E402

KINDS = ["inner", "leaf", "cold", "hot", "pair"]
MODES = {"cur": 0, "slotrec": 1, "pair": 2, "spec": 4, "blocks": 8, "fix": 64, "nofp": 128, "gf": 256, "gfptr": 512}


class View(ctypes.Structure):
    _fields_ = [("nodes", ctypes.c_void_p), ("n_nodes", ctypes.c_uint64), ("cold", ctypes.c_void_p),
                ("cold_slots", ctypes.c_uint64), ("hot", ctypes.c_void_p), ("hot_slots", ctypes.c_uint64),
                ("hot_limit", ctypes.c_uint32), ("aux_stride", ctypes.c_uint32), ("aux", ctypes.c_void_p)]


class SimOut(ctypes.Structure):
    _fields_ = [("req", ctypes.c_uint64 * 5), ("l1m", ctypes.c_uint64 * 5), ("l2m", ctypes.c_uint64 * 5),
                ("topics", ctypes.c_uint64), ("steps", ctypes.c_uint64), ("matches", ctypes.c_uint64),
                ("rounds", ctypes.c_uint64), ("probes_ok", ctypes.c_uint64), ("probes_fail", ctypes.c_uint64),
                ("table_visits", ctypes.c_uint64), ("plus_now", ctypes.c_uint64), ("plus_pop", ctypes.c_uint64),
                ("lit_inline", ctypes.c_uint64), ("reach_req", ctypes.c_uint64 * 5), ("reach_l2m", ctypes.c_uint64 * 5),
                ("wave_time", ctypes.c_double), ("wave_rounds", ctypes.c_double),
                ("waves", ctypes.c_uint64)]


def load_sim():
    so = os.path.join(ROOT, "tools", "sim", "libwalksim.so")
    src = os.path.join(ROOT, "tools", "sim", "walksim.cpp")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", src, "-o", so])
    lib = ctypes.CDLL(so)
    lib.sim_run.restype = ctypes.c_int
    return lib


def image(eng):
    v = View()
    lib = eng.lib
    lib.tm_debug_image.restype = ctypes.c_int
    rc = lib.tm_debug_image(eng.h, ctypes.byref(v))
    assert rc == 0, rc
    return v


def words(eng, tb, to):
    n = len(to) - 1
    lv = np.zeros(n, dtype=np.uint32)
    cap = int(to[-1]) + n + 1
    ids = np.zeros(cap, dtype=np.uint32)
    rc = eng.lib.tm_debug_words(eng.h, tb.ctypes.data_as(ctypes.c_void_p), to.ctypes.data_as(ctypes.c_void_p), n,
                                lv.ctypes.data_as(ctypes.c_void_p), ids.ctypes.data_as(ctypes.c_void_p),
                                ctypes.c_uint64(cap))
    assert rc == 0, rc
    dollar = np.array([tb[int(to[t])] == ord("$") if to[t + 1] > to[t] else 0 for t in range(n)], dtype=np.uint8)
    return lv, ids[: int(lv.sum())].copy(), dollar


def report(name, o, extra=None):
    t = o.topics
    d = {"layout": name, "topics": t, "steps": o.steps / t, "matches": o.matches / t}
    for k, nm in enumerate(KINDS):
        if o.req[k]:
            d[nm] = {"loads": round(o.req[k] / t, 2), "l1_miss": round(o.l1m[k] / t, 2),
                     "l2_miss": round(o.l2m[k] / t, 2)}
    d["loads"] = round(sum(o.req) / t, 2)
    d["l1_to_l2"] = round(sum(o.l1m) / t, 2)
    d["fabric"] = round(sum(o.l2m) / t, 2)
    d["l2_hit"] = round(1 - sum(o.l2m) / max(1, sum(o.l1m)), 3)
    d["probes_ok"] = round(o.probes_ok / t, 2)
    d["probes_fail"] = round(o.probes_fail / t, 2)
    d["table_visits"] = round(o.table_visits / t, 2)
    d["plus_now"] = round(o.plus_now / t, 2)
    d["plus_pop"] = round(o.plus_pop / t, 2)
    d["lit_inline"] = round(o.lit_inline / t, 2)
    d["node_loads_by_reach"] = {nm: [round(o.reach_req[k] / t, 2), round(o.reach_l2m[k] / t, 2)]
                                for k, nm in enumerate(["root", "plus_now", "plus_pop", "lit_inline", "lit_table"])}
    d["wave_rounds_per_topic"] = round(o.wave_rounds * o.waves / t, 3)
    d["model_cycles_per_topic"] = round(o.wave_time * o.waves / t, 1)
    if extra:
        d.update(extra)
    print(json.dumps(d), flush=True)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--filters", type=int, default=None)
    ap.add_argument("--topics", type=int, default=1_000_000, help="one XCD's share of the batch")
    ap.add_argument("--waves", type=int, default=6, help="waves per SIMD (occupancy; name+occN overrides)")
    ap.add_argument("--lat", default="120,350,1500", help="cycles of an L1 hit, an L2 hit, an L2 miss")
    ap.add_argument("--l2", type=int, default=4 << 20)
    ap.add_argument("--l1", type=int, default=32 << 10)
    ap.add_argument("--layouts", default="cur")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--bloom-hist", action="store_true", help="WIDE lookups by children count (no cache model)")
    ap.add_argument("--slice", type=int, default=-1,
                    help="with --sorted: 8 x --topics topics sorted as ONE batch (the global word-hash order), and "
                         "the walk of XCD range SLICE of them (the global sort hands each XCD a key-space slice)")
    ap.add_argument("--sorted", action="store_true",
                    help="topics in prefix order (lexicographic by word ids: the grouping of the walk's "
                         "word-hash order, presort 5)")
    a = ap.parse_args()
    cfg = W.CONFIGS[a.config]
    nf = a.filters or cfg["filters"]
    t0 = time.time()
    fb, fo = W.filters(a.config, n=nf)
    eng = Engine(device=-1, filters_hint=nf)
    for kv in a.opt:
        k, x = kv.split("=")
        eng.set_option(k, int(x))
    step = 5_000_000   # in chunks, with progress (a silent multi-minute build reads as a hang)
    n = len(fo) - 1
    for i in range(0, n, step):
        j = min(n, i + step)
        eng.insert_many(fb, fo[i:j + 1])
        print("# inserted %d / %d filters (%.0fs)" % (j, n, time.time() - t0), file=sys.stderr, flush=True)
    eng.commit()
    print("# built %d filters, %d nodes in %.1fs" % (eng.filter_count, eng.node_count, time.time() - t0),
          file=sys.stderr, flush=True)
    tb, to = W.topics(a.config, n=a.topics * (8 if a.slice >= 0 else 1), stream=0)
    lv, ids, dollar = words(eng, tb, to)
    if a.sorted:
        woff = np.zeros(len(lv) + 1, dtype=np.int64)
        woff[1:] = np.cumsum(lv)
        keys = [tuple(ids[woff[t]:woff[t + 1]][:8]) for t in range(len(lv))]
        order = sorted(range(len(lv)), key=lambda t: keys[t])
        if a.slice >= 0:
            n8 = len(order)
            order = order[n8 * a.slice // 8: n8 * (a.slice + 1) // 8]
        ids = np.concatenate([ids[woff[t]:woff[t + 1]] for t in order]).astype(np.uint32)
        lv, dollar = lv[order].copy(), dollar[order].copy()
    v = image(eng)
    lib = load_sim()

    if a.bloom_hist:
        h = (ctypes.c_uint64 * 48)()
        o = SimOut()
        p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        lib.sim_count(ctypes.byref(v), p(lv), p(ids), p(dollar), ctypes.c_uint32(len(lv)), ctypes.byref(o), h)
        n = len(lv)
        for b in range(16):
            if h[b]:
                print(json.dumps({"children_log2": b, "lookups": round(h[b] / n, 3), "bloom_pass": round(h[16 + b] / n, 3),
                                  "hits": round(h[32 + b] / n, 3),
                                  "false_pos": round((h[16 + b] - h[32 + b]) / n, 3)}))
    lat = (ctypes.c_double * 3)(*[float(x) for x in a.lat.split(",")])
    for name in [x for x in a.layouts.split(",") if x]:
        t1 = time.time()
        mode = 0
        occ = a.waves
        for part in name.split("+"):
            if part.startswith("occ"):
                occ = int(part[3:])
            elif part.startswith("gfmin"):   # gf: least literal children of a filtered node
                mode |= int(part[5:]) << 16
            elif part.startswith("gfbits"):   # gf: log2 words of the global filter (0: sized to ~8 % density)
                mode |= int(part[6:]) << 24
            elif part.startswith("div"):   # per-node block load: size >= div x edges
                mode |= int(part[3:]) << 8
            else:
                mode |= MODES[part]
        lanes = 32 * 4 * occ * 64
        o = SimOut()
        p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        lib.sim_run(ctypes.byref(v), p(lv), p(ids), p(dollar), ctypes.c_uint32(len(lv)), ctypes.c_uint32(lanes),
                    ctypes.c_uint32(4 * occ * 64), ctypes.c_uint64(a.l2), ctypes.c_uint64(a.l1), lat,
                    ctypes.c_int(mode), ctypes.byref(o))
        # time ~ (per-wave model time) x (topics per wave) / (waves in flight)
        report(name, o, {"waves_per_simd": occ, "sim_s": round(time.time() - t1, 1)})
    eng.close()


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
