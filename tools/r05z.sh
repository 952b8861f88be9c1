#!/bin/bash
# round 5: is the NIF path's latency tail CPU-quota throttling?  cgroup
# cpu.stat (nr_throttled, throttled_usec) around three latency runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05_z}
mkdir -p "$OUT"
stat() { echo "== $1"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null || cat /sys/fs/cgroup/cpu/cpu.stat 2>/dev/null || echo "no cpu.stat"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; }
for i in 1 2 3; do
  stat "before $i" >> "$OUT/cpustat.txt"
  timeout -k 10 200 python -u tools/bench_batcher_latency.py --rates 1e6,1e7 --deadlines 200 --eager 1 --eager-us 40 \
    > "$OUT/lat_$i.jsonl" 2>> "$OUT/latency.log" || exit $?
  stat "after $i" >> "$OUT/cpustat.txt"
done
