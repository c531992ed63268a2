"""Summarise rocprofv3 --pmc csv passes (gpurun_out/pmc/p*/) per kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].replace("gi::", "")
        c = row["Counter_Name"]
        acc[k][c] += float(row["Counter_Value"])
        cnt[k][c] += 1
for k in sorted(acc):
    if k.startswith("__amd"):
        continue
    d = acc[k]
    n = max(cnt[k].get("SQ_WAVES", 1), 1)
    print("==", k, "(dispatch-rows %d)" % n)
    for c in sorted(d):
        print("   %-24s %16.0f  per-dispatch %14.0f" % (c, d[c], d[c] / max(cnt[k][c], 1)))
