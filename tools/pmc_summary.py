"""Average PMC counter values per dispatch of each tm_* kernel over the
pass directories written by tools/pmc_passes.sh (one JSON object)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float)   # (dispatch, kernel, counter) -> value (summed over dimensions)
    for r in csv.DictReader(open(f)):
        m = re.search(r"tmx::(\w+)", r["Kernel_Name"])
        if not m:
            continue
        k = m.group(1)
        if "<true" in r["Kernel_Name"]:
            k += "<stats>"
        per[(r["Dispatch_Id"], k, r["Counter_Name"])] += float(r["Counter_Value"])
    for (disp, k, c), v in per.items():
        acc[k][c].append(v)
out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
print(json.dumps(out, indent=1, sort_keys=True))
