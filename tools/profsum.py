"""Summarize a rocprofv3 kernel_stats.csv: python tools/profsum.py <csv>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    name = r["Name"].split("(")[0].replace("tv::gpu::", "")
    print(f"{name:28s} calls={r['Calls']:>5} total_ms={int(r['TotalDurationNs'])/1e6:8.2f} "
          f"avg_us={float(r['AverageNs'])/1e3:9.1f} pct={float(r['Percentage']):5.1f}")
