#!/usr/bin/env python3
"""Compact per-kernel summary of a rocprofv3 kernel_stats.csv: short kernel name, calls,
total ms, average us, percent.  Usage: kstats.py <kernel_stats.csv> [top]"""
import csv
import re
import sys


def short(name: str) -> str:
    n = name.replace("tv::gpu::(anonymous namespace)::", "").replace("tv::gpu::", "")
    n = re.sub(r"\(.*", "", n)
    return n[:60]


rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 15
for r in rows[:top]:
    print(f"{short(r['Name']):60s} calls={int(r['Calls']):6d} total_ms={int(r['TotalDurationNs']) / 1e6:9.2f} "
          f"avg_us={float(r['AverageNs']) / 1e3:9.1f} pct={float(r['Percentage']):5.1f}")
