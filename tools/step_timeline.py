"""One steady-state step's kernel timeline from a rocprofv3 rocpd database.
usage: python tools/step_timeline.py <db> [which_step_from_end=6]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
back = int(sys.argv[2]) if len(sys.argv) > 2 else 6
rows = c.execute("select name, start, end from kernels order by start").fetchall()
idx = [i for i, r in enumerate(rows) if "swap_k" in r[0] or "conv_fwd_in_swap" in r[0]]  # the step's first kernel
i0, i1 = idx[-back], idx[-back + 1]
t0 = rows[i0][1]
busy = 0
for r in rows[i0:i1]:
    d = (r[2] - r[1]) / 1e3
    busy += d
    print(f"{(r[1] - t0) / 1e3:8.1f} {(r[2] - t0) / 1e3:8.1f} {d:8.2f}  {r[0][:100]}")
print(f"kernel-sum {busy:.1f} us, step span {(rows[i1][1] - t0) / 1e3:.1f} us")
