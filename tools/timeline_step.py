"""Timeline view of the last training step(s) in a rocprofv3 rocpd .db (``--kernel-trace``).

    python tools/timeline_step.py run.db STEP_MS [NSTEPS] [--list]

Takes the kernels of the last NSTEPS·STEP_MS of the trace and reports, per HIP stream (queue),
busy time; the union of all streams' busy time (GPU occupied by >= 1 kernel); the idle gaps
between kernels on the critical (busiest) stream; and with ``--list`` the kernel sequence of one
step with per-kernel durations, so the critical path of a step can be read off directly."""
import collections
import sqlite3
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    db, step_ms = args[0], float(args[1])
    nsteps = int(args[2]) if len(args) > 2 else 1
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    ki = {n: i for i, n in enumerate(cols)}
    rows = c.execute("select * from kernels").fetchall()
    qcol = next((n for n in ("queue_id", "stream_id", "queue", "stream") if n in ki), None)
    name_col = "name" if "name" in ki else [n for n in cols if "name" in n][0]
    tmax = max(r[ki["end"]] for r in rows)
    t0 = tmax - nsteps * step_ms * 1e6
    rows = sorted((r for r in rows if r[ki["start"]] >= t0), key=lambda r: r[ki["start"]])
    per_q = collections.defaultdict(float)
    ivs = []
    for r in rows:
        s, e = r[ki["start"]], r[ki["end"]]
        q = r[ki[qcol]] if qcol else 0
        per_q[q] += (e - s) / 1e6
        ivs.append((s, e))
    # union of busy intervals
    union, cs, ce = 0.0, None, None
    for s, e in sorted(ivs):
        if cs is None:
            cs, ce = s, e
        elif s <= ce:
            ce = max(ce, e)
        else:
            union += (ce - cs) / 1e6
            cs, ce = s, e
    if cs is not None:
        union += (ce - cs) / 1e6
    span = (rows[-1][ki["end"]] - rows[0][ki["start"]]) / 1e6 if rows else 0.0
    print(f"window {nsteps} step(s) x {step_ms:.3f} ms; kernels {len(rows)}; span {span:.3f} ms")
    print(f"GPU busy (union of streams) {union / nsteps:.3f} ms/step; idle {max(0.0, span - union) / nsteps:.3f} ms/step")
    for q, t in sorted(per_q.items(), key=lambda x: -x[1]):
        print(f"  queue {q}: busy {t / nsteps:.3f} ms/step")
    crit = max(per_q, key=per_q.get) if per_q else None
    gaps = []
    last_e = None
    for r in rows:
        if qcol and r[ki[qcol]] != crit:
            continue
        if last_e is not None:
            gaps.append((r[ki["start"]] - last_e) / 1e3)
        last_e = r[ki["end"]]
    if gaps:
        big = [g for g in gaps if g > 5.0]
        print(f"critical queue {crit}: {len(gaps)} gaps, total {sum(gaps) / 1e3 / nsteps:.3f} ms/step, "
              f">5us: {len(big)} totalling {sum(big) / 1e3 / nsteps:.3f} ms/step")
    if "--list" in sys.argv:
        t1 = tmax - step_ms * 1e6
        for r in rows:
            if r[ki["start"]] < t1:
                continue
            q = r[ki[qcol]] if qcol else 0
            print(f"{(r[ki['start']] - t1) / 1e3:9.1f} us  q{q}  {(r[ki['end']] - r[ki['start']]) / 1e3:8.1f} us  "
                  f"{str(r[ki[name_col]])[:110]}")


if __name__ == "__main__":
    main()
