"""Aggregate a rocprofv3 counter_collection.csv per kernel: python tools/pmcsum.py <csv> [kernel-substr]"""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
calls = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("tv::gpu::", "")
    if len(sys.argv) > 2 and sys.argv[2] not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    calls[k].add(r["Dispatch_Id"])
for k, c in sorted(agg.items(), key=lambda x: -x[1].get("SQ_BUSY_CYCLES", x[1].get("SQ_WAVES", 0))):
    n = len(calls[k])
    print(k, f"dispatches={n}", " ".join(f"{name}={v / n:.4g}" for name, v in sorted(c.items())))
