"""PMC counters of one kernel per dispatch, in dispatch order, from a
rocprofv3 --pmc pass (run_counter_collection.csv): for bench runs that time
several variants in one process (bench.py --ab-opt), where the per-kernel
average of tools/pmc_summary.py would mix them.  Prints one JSON line per
dispatch of the kernel (tmx::<name>), with the counters summed over their
dimensions, and the topics-normalised values when --topics is given.

  python tools/pmc_sequence.py gpurun_out/x/pmc/tcctlb tm_walk_queue --topics 8000000
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("--topics", type=int, default=0)
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))
    name = {}
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"tmx::(\w+)", r["Kernel_Name"])
            if not m or m.group(1) != a.kernel or "<true" in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            name[d] = r["Kernel_Name"]
    for i, d in enumerate(sorted(per)):
        row = {"seq": i, "dispatch": d, "counters": dict(per[d])}
        if a.topics:
            row["per_topic"] = {k: v / a.topics for k, v in per[d].items()}
        print(json.dumps(row))


if __name__ == "__main__":
    main()
