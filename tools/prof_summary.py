"""Summarise a rocprofv3 rocpd SQLite database: per-kernel totals, one row per
(kernel, grid) -- a kernel launched at several mesh levels gets one row per
level (their grids differ), so each row's average is one layer's duration."""
import sqlite3
import sys

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(end-start), sum(end-start), min(end-start), max(end-start), "
                 "grid_x, grid_y from kernels group by name, grid_x, grid_y "
                 "order by sum(end-start) desc").fetchall()
tot = sum(r[3] for r in rows)
print(f"{'share':>6} {'calls':>6} {'avg_us':>9} {'min_us':>9} {'max_us':>9} {'grid':>12}  kernel")
for r in rows[:top]:
    grid = f"{r[6]}x{r[7]}"
    print(f"{r[3] / tot * 100:5.1f}% {r[1]:6d} {r[2] / 1e3:9.2f} {r[4] / 1e3:9.2f} {r[5] / 1e3:9.2f} {grid:>12}  {r[0][:110]}")
print(f"total kernel time {tot / 1e6:.3f} ms over {sum(r[1] for r in rows)} dispatches")
