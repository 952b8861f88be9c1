#!/bin/bash
# round 5: HIP API trace of the 10M publishes/s latency run (4 lanes): which
# HIP call inside the engine's enqueue blocks for milliseconds?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_ah}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/bench_batcher_latency.py --rates 1e7 --deadlines 200 --eager 1 --eager-us 40 --lanes 4 \
  > "$OUT/lat.jsonl" 2> "$OUT/lat.log" || exit $?
python3 - "$OUT" > "$OUT/long_calls.txt" <<'PY'
import csv, sys, glob
out = sys.argv[1]
f = glob.glob(out + "/trace/*hip_api_trace.csv")[0]
rows = []
for r in csv.DictReader(open(f)):
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    rows.append((d, r["Function"], r["Thread_Id"], int(r["Start_Timestamp"])))
t0 = min(x[3] for x in rows)
rows.sort(reverse=True)
for d, fn, th, s in rows[:60]:
    print("%9.1f us  %-32s thread %s  at %.1f ms" % (d / 1e3, fn, th, (s - t0) / 1e6))
PY
