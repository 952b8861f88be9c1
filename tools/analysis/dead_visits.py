"""Driver of tools/analysis/dead_visits.c: dump a config's filters and topics
and run the analysis (how many walk visits a subtree summary could skip).
    python tools/analysis/dead_visits.py [config] [n_topics]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from emqx_amd import workload as W  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
nt = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
src = os.path.join(ROOT, "tools", "analysis", "dead_visits.c")
exe = "/tmp/dead_visits"
subprocess.check_call(["gcc", "-O2", "-o", exe, src])


def dump(path, buf, off):
    with open(path, "wb") as f:
        np.array([len(off) - 1], dtype=np.uint64).tofile(f)
        np.asarray(off, dtype=np.uint64).tofile(f)
        np.asarray(buf[: int(off[-1])], dtype=np.uint8).tofile(f)


dump("/tmp/dv_f.bin", *W.filters(cfg))
dump("/tmp/dv_t.bin", *W.topics(cfg, n=nt))
print(subprocess.check_output([exe, "/tmp/dv_f.bin", "/tmp/dv_t.bin"]).decode())
