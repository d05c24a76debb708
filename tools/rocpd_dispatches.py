"""Per-dispatch listing of a rocprofv3 rocpd .db: the last N kernel dispatches in launch order
(name, grid, workgroup, duration µs) — for mapping one iteration's launches to layers."""
import sqlite3
import sys

db, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 100
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
ki = {k: i for i, k in enumerate(cols)}
rows = sorted(c.execute("select * from kernels").fetchall(), key=lambda r: r[ki["start"]])[-n:]
name_col = "name" if "name" in ki else [k for k in cols if "name" in k][0]


def g(r, *keys):
    for k in keys:
        if k in ki:
            return r[ki[k]]
    return "?"


print("columns:", ",".join(cols))
for r in rows:
    grid = (g(r, "grid_size_x", "grid_x", "grid_size"), g(r, "grid_size_y", "grid_y"), g(r, "grid_size_z", "grid_z"))
    wg = (g(r, "workgroup_size_x", "workgroup_x", "workgroup_size"),)
    print(f"{(r[ki['end']] - r[ki['start']]) / 1e3:9.1f} us  grid={grid} wg={wg}  {str(r[ki[name_col]])[:70]}")
