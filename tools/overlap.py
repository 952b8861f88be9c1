"""Kernel overlap in a rocprofv3 kernel trace (run_kernel_trace.csv): for the
last N walk launches, how long the other match-pipeline kernels ran beside a
walk (on another queue) versus serially.

    python tools/overlap.py gpurun_out/<tag>/prof3/run_kernel_trace.csv [N] [SKIP]

N walks after the first SKIP (default 2: bench.py's two untimed sizing
passes), i.e. the warm-up and timed steps (the serial roof steps follow).
Prints one JSON object: per kernel family the summed duration, the part of
it that overlapped another walk, and the wall time the pipeline spanned.
"""
import csv
import json
import sys


def family(name):
    for k in ("tm_walk_queue", "tm_tokenize", "tm_copy_out", "tm_scan"):
        if k in name:
            return k
    return None


def main(path, last=20, skip=2):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            fam = family(r["Kernel_Name"])
            if fam:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam, r["Queue_Id"]))
    rows.sort()
    walks = [r for r in rows if r[2] == "tm_walk_queue"][skip:skip + last]
    if not walks:
        print(json.dumps({"error": "no walks"}))
        return
    t0, t1 = walks[0][0], walks[-1][1]
    win = [r for r in rows if r[1] > t0 and r[0] < t1]
    out = {"walks": len(walks), "wall_ms": (t1 - t0) / 1e6, "families": {}}
    for fam in ("tm_walk_queue", "tm_tokenize", "tm_scan", "tm_copy_out"):
        tot = ov = 0
        for s, e, f, q in win:
            if f != fam:
                continue
            tot += e - s
            for ws, we, _, wq in walks:
                if (ws, we) != (s, e):
                    ov += max(0, min(e, we) - max(s, ws))
        out["families"][fam] = {"sum_ms": tot / 1e6, "beside_walk_ms": ov / 1e6}
    # busy union of all pipeline kernels
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    out["busy_ms"] = busy / 1e6
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20, int(sys.argv[3]) if len(sys.argv) > 3 else 2)
