"""Per-kernel duration summary from a rocprofv3 rocpd database (rocprofv3 -d DIR -o run)."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
pat = sys.argv[2] if len(sys.argv) > 2 else "%"
rows = db.execute("select name, count(*), avg(duration)/1000.0, min(duration)/1000.0, sum(duration)/1000.0 from kernels "
                  "where name like ? group by name order by sum(duration) desc limit 40", (pat,)).fetchall()
print(f"{'calls':>6} {'avg_us':>9} {'min_us':>9} {'total_us':>10}  kernel")
for name, n, avg, mn, tot in rows:
    print(f"{n:6d} {avg:9.1f} {mn:9.1f} {tot:10.1f}  {name[:120]}")
