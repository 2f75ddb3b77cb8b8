"""One steady-state data-parallel step's kernel timeline (rank 0) from a
rocprofv3 rocpd database, with every gap between consecutive kernels (host
time between the three graph replays, the all-reduce joins) and the totals.
usage: python tools/dp_timeline.py <db> [which_step_from_end=6]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
back = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows = c.execute("select name, start, end from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if "step_begin_k" in r[0]]
# data-parallel steps end with their own Adam launch (adam_k); pick the
# back-th such step from the last one
dp = [(a, b) for a, b in zip(idx, idx[1:]) if any("adam_k" in r[0] for r in rows[a:b])]
i0, i1 = dp[-back]
t0 = rows[i0][1]
busy = gaps = 0.0
prev_end = None
for r in rows[i0:i1]:
    d = (r[2] - r[1]) / 1e3
    gap = (r[1] - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += d
    gaps += max(gap, 0.0)
    mark = f"  <-- gap {gap:7.1f} us" if gap > 1.0 else ""
    print(f"{(r[1] - t0) / 1e3:8.1f} {(r[2] - t0) / 1e3:8.1f} {d:8.2f}  {r[0][:90]}{mark}")
    prev_end = r[2]
span = (rows[i1][1] - t0) / 1e3
print(f"kernel-sum {busy:.1f} us, gaps {gaps + (rows[i1][1] - prev_end) / 1e3:.1f} us "
      f"(last gap to the next step {(rows[i1][1] - prev_end) / 1e3:.1f} us), step span {span:.1f} us")
