"""Per-kernel HBM bytes of one training step from tools/pmc_step_bytes.sh CSV passes."""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]


def load(counter):
    path = glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True)
    rows = [r for p in path for r in csv.DictReader(open(p))]
    rows.sort(key=lambda r: int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))))
    return rows


def one_step(rows):
    idx = [i for i, r in enumerate(rows) if "k_sgd" in r["Kernel_Name"]]
    if len(idx) < 2:
        return rows
    return rows[idx[-2] + 1: idx[-1] + 1]


tot = {}
per = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(int)
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = one_step(load(c))
    t = 0.0
    for r in rows:
        v = float(r["Counter_Value"]) * 1024.0  # KB -> bytes
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:60]
        per[name][c] += v
        if c == "FETCH_SIZE":
            cnt[name] += 1
        t += v
    tot[c] = t
print(f"one step: fetched {tot['FETCH_SIZE'] / 1e9:.2f} GB, written {tot['WRITE_SIZE'] / 1e9:.2f} GB, "
      f"total {(tot['FETCH_SIZE'] + tot['WRITE_SIZE']) / 1e9:.2f} GB")
for name, d in sorted(per.items(), key=lambda x: -(x[1]["FETCH_SIZE"] + x[1]["WRITE_SIZE"])):
    print(f"  {(d['FETCH_SIZE'] + d['WRITE_SIZE']) / 1e9:7.3f} GB  (rd {d['FETCH_SIZE'] / 1e9:6.3f} wr "
          f"{d['WRITE_SIZE'] / 1e9:6.3f})  n={cnt[name]:4d}  {name}")
