"""Summarise a rocprofv3 --marker-trace CSV (roctx ranges pushed by bigdl.utils.tracing with
bigdl.roctx=1): per range name, count and total / mean host-side duration.  Usage:
    python tools/marker_summary.py gpurun_out/r2/prof_mark [n_steps]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
files = glob.glob(os.path.join(root, "**", "*marker_api_trace.csv"), recursive=True)
if not files:
    print("no marker trace CSV under", root)
    sys.exit(1)
agg = collections.defaultdict(lambda: [0, 0.0])
for f in files:
    for row in csv.DictReader(open(f)):
        name = row.get("Function") or row.get("Name") or row.get("Message") or "?"
        try:
            dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
        except (KeyError, ValueError):
            continue
        a = agg[name]
        a[0] += 1
        a[1] += dur
print(f"{'range':28s} {'count':>6s} {'total ms':>10s} {'ms/step':>9s} {'mean ms':>9s}")
for name, (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{name[:28]:28s} {n:6d} {tot:10.3f} {tot / steps:9.3f} {tot / n:9.3f}")
