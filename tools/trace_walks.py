"""Walk durations in dispatch order from a rocprofv3 kernel trace
(run_kernel_trace.csv): one line per tm_walk_queue launch with its duration
and the gap since the previous pipeline kernel ended, grouped into runs of
consecutive launches whose grid and duration class agree -- for in-process
A/Bs (bench.py --ab-opt), where the variants' walks follow each other.

    python tools/trace_walks.py gpurun_out/<tag>/prof/run_kernel_trace.csv
"""
import csv
import json
import sys


def main(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    out = []
    for i, (a, b, name) in enumerate(rows):
        if "tm_walk_queue" not in name:
            continue
        prev_end = max((r[1] for r in rows[max(0, i - 8):i] if r[1] <= a), default=a)
        out.append({"i": len(out), "ms": round((b - a) / 1e6, 4), "gap_us": round((a - prev_end) / 1e3, 1),
                    "kernel": name.split("(")[0][:60]})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    main(sys.argv[1])
