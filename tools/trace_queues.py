#!/usr/bin/env python3
"""Per-queue busy time and kernel mix of a rocprofv3 kernel_trace.csv (time window = the last
N ms of the trace).  Usage: trace_queues.py <kernel_trace.csv> [window_ms]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
win = float(sys.argv[2]) if len(sys.argv) > 2 else 0
end = max(int(r["End_Timestamp"]) for r in rows)
t0 = end - win * 1e6 if win else min(int(r["Start_Timestamp"]) for r in rows)
busy = collections.defaultdict(list)
mix = collections.defaultdict(lambda: collections.Counter())
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e < t0:
        continue
    q = (r["Queue_Id"], r.get("Stream_Id", ""))
    busy[q].append((max(s, t0), e))
    m = re.search(r"(k_\w+|__amd_\w+)", r["Kernel_Name"])
    mix[q][m.group(1) if m else r["Kernel_Name"][:30]] += (e - max(s, t0)) / 1e6


def union(iv):
    iv.sort()
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot


span = (end - t0) / 1e6
print(f"window {span:.1f} ms")
for q, iv in sorted(busy.items(), key=lambda x: -union(list(x[1]))):
    u = union(list(iv)) / 1e6
    top = ", ".join(f"{k} {v:.0f}" for k, v in mix[q].most_common(4))
    print(f"queue {q}: busy {u:.1f} ms ({100 * u / span:.0f}%), {len(iv)} kernels: {top}")
