"""Dev: per-kernel duration summary of a rocprofv3 rocpd database (default output format).
Usage: kstats.py results.db [last_n]  -- last_n: only the last N dispatches (e.g. one graph-replay
phase); prints count, mean / median us per kernel name and the mean gap between dispatches."""
import sqlite3
import statistics
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, start, end from kernels order by start").fetchall()
if len(sys.argv) > 2:
    rows = rows[-int(sys.argv[2]):]
by = {}
for name, s, e in rows:
    short = name.replace("(anonymous namespace)::", "").split("(")[0][:90]
    by.setdefault(short, []).append((e - s) / 1e3)
gaps = [(rows[i + 1][1] - rows[i][2]) / 1e3 for i in range(len(rows) - 1)]
span = (rows[-1][2] - rows[0][1]) / 1e3
print(f"{len(rows)} dispatches over {span:.1f} us; mean gap {statistics.mean(gaps):.2f} us, "
      f"median gap {statistics.median(gaps):.2f} us")
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    print(f"{len(v):6d}  mean {statistics.mean(v):8.2f}  median {statistics.median(v):8.2f}  "
          f"total {sum(v):10.1f}  {k}")
