"""Per-launch HBM traffic of the dominant kernel from a PMC pass directory
(tools/pmc_passes.sh): FETCH_SIZE + WRITE_SIZE of tm_walk_queue, as the
`roofline.traffic` figure bench.py reports.

Units and corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section):
FETCH_SIZE/WRITE_SIZE are in KB.  The guide's x2 correction is for wide
coalesced streaming reads; the walk's reads are random 16 B gathers, which
the gather microbenchmark calibrates at exactly one TCC_EA0_RDREQ = 64 B of
FETCH_SIZE per L2-missing access (profiles/r02_gather/gather_pmc.json:
33.5M accesses over a 4 GiB table -> 33.5M EA read requests, 63.9 B of
FETCH_SIZE each), so FETCH_SIZE is taken as is.

usage: python tools/traffic.py gpurun_out/pmc_x profiles/traffic_c3.json
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_src_sha():
    """hash of the walk's sources: bench.py reports the traffic only for the same kernel"""
    h = hashlib.sha256()
    for f in ("kernels.hip", "image.h", "kernels.h"):
        h.update(open(os.path.join(ROOT, "emqx_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:16]


def launches(src, counter):
    """the counter of every tm_walk_queue dispatch (not the stats variant),
    in dispatch order, summed over its dimensions"""
    import csv
    import glob
    import re
    per = {}
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            m = re.search(r"tmx::(\w+)", r["Kernel_Name"])
            if not m or m.group(1) != "tm_walk_queue" or "<true" in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            d = int(r["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    return [per[d] for d in sorted(per)]


def headline(src, counter):
    """mean over the bench's full-size launches: a bench process may also walk
    smaller batches (the weak-scaling 1M-topic leg), which the per-kernel
    average of summary.json would mix in"""
    v = launches(src, counter)
    top = max(v)
    big = [x for x in v if x >= 0.5 * top]
    return sum(big) / len(big)


src, dst = sys.argv[1], sys.argv[2]
w = {c: headline(src, c) for c in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum")}
log = open(src + "/fetch/log.txt").read().splitlines()
line = next((json.loads(x) for x in log if x.startswith("{")), None)
cfg = line["config"] if line else None
rev = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip() or None
out = {
    "kernel": "tm_walk_queue",
    "config": cfg,
    "fetch_bytes_per_launch": w["FETCH_SIZE"] * 1024.0,
    "write_bytes_per_launch": w["WRITE_SIZE"] * 1024.0,
    "traffic_bytes_per_launch": (w["FETCH_SIZE"] + w["WRITE_SIZE"]) * 1024.0,
    "l2_hit_rate": w["TCC_HIT_sum"] / (w["TCC_HIT_sum"] + w["TCC_MISS_sum"]),
    "ea_read_requests_per_launch": w.get("TCC_EA0_RDREQ_sum"),
    "correction": "none: random 16 B gathers, 1 EA read request = 64 B of FETCH_SIZE per missed access "
                  "(profiles/r02_gather/gather_pmc.json)",
    "source": src,
    "build": rev,
    "kernel_src_sha": kernel_src_sha(),
}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
