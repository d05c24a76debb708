"""GPU busy time of a rocprofv3 rocpd .db: the union of kernel intervals (any stream) over the
window of the last LAST_MS milliseconds of the trace, against that window's wall time.  A step
whose busy fraction is well below 1 is host (dispatch) bound.

    python tools/rocpd_busy.py run.db [last_ms] [steps_in_window]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    steps = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
    c = sqlite3.connect(db)
    rows = c.execute("select start, \"end\" from kernels").fetchall()
    if not rows:
        print("no kernels")
        return
    tmax = max(e for _, e in rows)
    t0 = tmax - last_ms * 1e6 if last_ms > 0 else min(s for s, _ in rows)
    iv = sorted((max(s, t0), e) for s, e in rows if e > t0)
    busy, cur_s, cur_e = 0.0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    wall = tmax - t0
    ksum = sum(e - s for s, e in iv)
    print(f"window {wall / 1e6:.3f} ms, {len(iv)} kernels; busy {busy / 1e6:.3f} ms ({100 * busy / wall:.1f} %), "
          f"kernel sum {ksum / 1e6:.3f} ms; per step: wall {wall / 1e6 / steps:.3f} busy {busy / 1e6 / steps:.3f} "
          f"kernels {len(iv) / steps:.1f}")


if __name__ == "__main__":
    main()
