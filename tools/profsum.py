"""Summarize rocprofv3 output.

    python tools/profsum.py <run_kernel_stats.csv>                 # whole run (rocprof stats)
    python tools/profsum.py <run_kernel_trace.csv> --skip 0.5      # trace, drop the first half
                                                                   # of the timeline (clock ramp,
                                                                   # warm-up steps)
"""
import argparse
import csv
from collections import defaultdict


def short(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").split("(")[0].replace("tv::gpu::", "").replace("tv::ops::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--skip", type=float, default=0.0, help="fraction of the trace timeline to drop")
    ap.add_argument("--top", type=int, default=0)
    ap.add_argument("--seq", default="", help="KERNEL:N -- mean duration of that kernel's calls by call index mod N "
                    "(e.g. the rounds of an iterated kernel)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    if a.seq:
        name, n = a.seq.rsplit(":", 1)
        n = int(n)
        calls = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                       for r in rows if short(r.get("Kernel_Name", "")).endswith(name))
        for i in range(n):
            d = [t for j, (_, t) in enumerate(calls) if j % n == i]
            print(f"{name}[{i} mod {n}] calls={len(d)} avg_us={sum(d) / max(1, len(d)) / 1e3:.1f}")
    if "Calls" in rows[0]:
        out = [(short(r["Name"]), int(r["Calls"]), int(r["TotalDurationNs"])) for r in rows]
    else:
        t0 = min(int(r["Start_Timestamp"]) for r in rows)
        t1 = max(int(r["End_Timestamp"]) for r in rows)
        cut = t0 + a.skip * (t1 - t0)
        agg = defaultdict(lambda: [0, 0])
        for r in rows:
            if int(r["Start_Timestamp"]) < cut:
                continue
            k = agg[short(r["Kernel_Name"])]
            k[0] += 1
            k[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        out = [(n, c, t) for n, (c, t) in agg.items()]
    if a.seq:
        return
    out.sort(key=lambda x: -x[2])
    tot = sum(t for _, _, t in out) or 1
    for n, c, t in out[: a.top or None]:
        print(f"{n:28s} calls={c:>5} total_ms={t / 1e6:8.2f} avg_us={t / max(c, 1) / 1e3:9.1f} pct={100 * t / tot:5.1f}")


if __name__ == "__main__":
    main()
