"""Host-vs-device lag per kernel from a rocprofv3 rocpd .db recorded with --kernel-trace --hip-trace:
for each kernel of the last N steps, the time from its launch API call returning on the host to the
kernel starting on the device.  Small lag right before a device-idle gap = the host was late (host
bound there); large lag = the kernel sat queued behind earlier work (device bound).

    python tools/launch_lag.py run.db STEP_MS [NSTEPS]"""
import sqlite3
import sys


def main():
    db, step_ms = sys.argv[1], float(sys.argv[2])
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    kc = [r[1] for r in c.execute("pragma table_info(kernels)")]
    rc = [r[1] for r in c.execute("pragma table_info(regions)")] if "regions" in tabs else []
    print("kernels cols:", kc)
    print("regions cols:", rc)
    kid = next((n for n in ("correlation_id", "corr_id") if n in kc), None)
    rid = next((n for n in ("correlation_id", "corr_id") if n in rc), None)
    if not (kid and rid):
        print("no correlation ids; cannot pair launches")
        return
    K = c.execute(f"select start, end, {kid}, name, {'queue_id' if 'queue_id' in kc else 'stream_id'} from kernels").fetchall()
    R = {}
    for r in c.execute(f"select start, end, {rid}, name from regions").fetchall():
        if "Launch" in r[3] or "launch" in r[3]:
            R[r[2]] = r
    # diagnostics: how a few kernels pair with their launch calls
    for k in sorted(K, key=lambda k: k[0])[-5:]:
        r = R.get(k[2])
        print("sample kernel", k[2], k[3][:40], "start", k[0], "| launch", r[3][:30] if r else None,
              r[0] if r else None, r[1] if r else None)
    names = {}
    for r in c.execute("select name from regions").fetchall():
        names[r[0]] = names.get(r[0], 0) + 1
    print("region names:", sorted(names.items(), key=lambda x: -x[1])[:12])
    tmax = max(k[1] for k in K)
    t0 = tmax - nsteps * step_ms * 1e6
    K = sorted((k for k in K if k[0] >= t0), key=lambda k: k[0])
    lags = []
    prev_end = None
    for k in K:
        r = R.get(k[2])
        lag = (k[0] - r[1]) / 1e3 if r else float("nan")
        gap = (k[0] - prev_end) / 1e3 if prev_end is not None else 0.0
        prev_end = max(prev_end or 0, k[1])
        lags.append((lag, gap, (k[1] - k[0]) / 1e3, k[4], k[3][:70]))
    host_late = [l for l in lags if l[1] > 10 and l[0] < 20]
    print(f"{len(lags)} kernels; gaps > 10 us: {sum(1 for l in lags if l[1] > 10)} "
          f"({sum(l[1] for l in lags if l[1] > 10):.0f} us), of which host-late (lag < 20 us): {len(host_late)} "
          f"({sum(l[1] for l in host_late):.0f} us)")
    for l in sorted(lags, key=lambda l: -l[1])[:30]:
        print(f"gap {l[1]:8.1f} us  lag {l[0]:8.1f} us  dur {l[2]:7.1f} q{l[3]}  {l[4]}")


if __name__ == "__main__":
    main()
