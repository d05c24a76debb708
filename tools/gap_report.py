"""Largest idle gaps on the busiest HIP queue in the last N steps of a rocprofv3 rocpd .db, with the
kernels on either side and what the other queues were running meanwhile.

    python tools/gap_report.py run.db STEP_MS [NSTEPS] [TOP]"""
import collections
import sqlite3
import sys


def main():
    db, step_ms = sys.argv[1], float(sys.argv[2])
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 30
    c = sqlite3.connect(db)
    rows = c.execute("select name, queue_id, start, end from kernels order by start").fetchall()
    tmax = max(r[3] for r in rows)
    rows = [r for r in rows if r[2] >= tmax - nsteps * step_ms * 1e6]
    byq = collections.defaultdict(list)
    for r in rows:
        byq[r[1]].append(r)
    q = max(byq, key=lambda k: sum(r[3] - r[2] for r in byq[k]))
    main_q = byq[q]
    others = [r for r in rows if r[1] != q]
    gaps = []
    for a, b in zip(main_q, main_q[1:]):
        g = b[2] - a[3]
        if g > 0:
            gaps.append((g, a, b))
    gaps.sort(key=lambda x: -x[0])
    tot = sum(g for g, _, _ in gaps) / 1e6 / nsteps
    print(f"queue {q}: {len(main_q) / nsteps:.0f} kernels/step, idle {tot:.3f} ms/step")
    by_pair = collections.Counter()
    for g, a, b in gaps:
        by_pair[(a[0].split("(")[0][:60], b[0].split("(")[0][:60])] += g
    print("idle by (before -> after) kernel pair, ms/step:")
    for (x, y), g in by_pair.most_common(top):
        print(f"  {g / 1e6 / nsteps:7.3f}  {x}  ->  {y}")
    print("largest gaps:")
    for g, a, b in gaps[:top]:
        ov = [o[0].split("(")[0][:40] for o in others if o[2] < b[2] and o[3] > a[3]]
        print(f"  {g / 1e3:8.1f} us  {a[0].split('(')[0][:50]} -> {b[0].split('(')[0][:50]}  | other q: {ov[:3]}")


if __name__ == "__main__":
    main()
