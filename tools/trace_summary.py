"""Summarize a rocprofv3 kernel trace (run_kernel_trace.csv): per-launch durations in order
(kernels >= 0.05 ms) and totals per kernel name.

    python tools/trace_summary.py <trace dir or csv> [min_ms]"""
import collections
import csv
import os
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = os.path.join(path, "run_kernel_trace.csv")
min_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
tot = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    name = r["Kernel_Name"].replace("oap::kern::(anonymous namespace)::", "")
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    tot[name[:90]][0] += 1
    tot[name[:90]][1] += dur
    if dur >= min_ms:
        print(f"{dur:8.3f}  {name[:100]}")
print("\n  calls   total_ms  kernel")
for name, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
    print(f"{c:7d} {t:10.3f}  {name}")
