"""Per-kernel summary (calls, average / total duration, share) of a rocprofv3 SQLite output
(`rocprofv3 --kernel-trace` without --output-format csv).  Usage: python tools/prof_db.py <dir|db>"""
import glob
import os
import sqlite3
import sys

p = sys.argv[1]
db = p if p.endswith(".db") else sorted(glob.glob(os.path.join(p, "**", "*.db"), recursive=True))[0]
rows = sqlite3.connect(db).execute(
    "select name, count(*), avg(duration), sum(duration) from kernels group by name order by 4 desc").fetchall()
tot = sum(r[3] for r in rows)
print(f"{'kernel':80s} {'calls':>6s} {'avg_us':>10s} {'total_ms':>10s} {'pct':>6s}")
for name, n, avg, s in rows:
    print(f"{name[:80]:80s} {n:6d} {avg / 1e3:10.1f} {s / 1e6:10.3f} {s / tot * 100:6.1f}")
