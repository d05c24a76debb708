"""Summarise a rocprofv3 rocpd .db: per-kernel total/avg time, grouped; writes markdown."""
import sqlite3, sys, re, collections
db = sys.argv[1]; steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
rows = c.execute("select * from kernels").fetchall()
ki = {n: i for i, n in enumerate(cols)}
import os
last_ms = float(os.environ.get('LAST_MS', '0'))
if last_ms > 0:
    tmax = max(r[ki['end']] for r in rows)
    rows = [r for r in rows if r[ki['start']] >= tmax - last_ms * 1e6]
name_col = 'name' if 'name' in ki else [n for n in cols if 'name' in n][0]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    nm = r[ki[name_col]]; dur = (r[ki['end']] - r[ki['start']]) / 1e6
    agg[nm][0] += 1; agg[nm][1] += dur
tot = sum(v[1] for v in agg.values())
def cat(n):
    n2 = n.lower()
    for k, pats in [("conv", ["conv", "igemm", "implicit", "gemm", "cijk", "xdl"]), ("bn", ["batch_norm", "batchnorm", "bn_", "miopenbatch"]),
                    ("elementwise", ["elementwise", "vectorized", "relu", "add", "clamp"]), ("reduce", ["reduce"]), ("pool", ["pool"])]:
        if any(p in n2 for p in pats): return k
    return "other"
cats = collections.defaultdict(float)
for n, (cnt, t) in agg.items(): cats[cat(n)] += t
print(f"total kernel time {tot:.1f} ms over {steps} steps = {tot/steps:.2f} ms/step")
for k, v in sorted(cats.items(), key=lambda x: -x[1]): print(f"  {k:12s} {v/steps:8.2f} ms/step  {100*v/tot:5.1f}%")
print("top kernels:")
for n, (cnt, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"  {t/steps:8.3f} ms/step  n={cnt:6d}  {n[:150]}")
