"""Kernel sequence of a window of a rocprofv3 rocpd database (development tool):
python tools/rocpd_timeline.py run_results.db FIRST COUNT  -> name, grid, duration, gap to the previous end."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
first, count = int(sys.argv[2]), int(sys.argv[3])
cols = [r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")]
grid = "d.grid_size_x" if "grid_size_x" in cols else "0"
q = (f"select s.kernel_name, d.start, d.end, {grid} from rocpd_kernel_dispatch d "
     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start")
rows = list(c.execute(q))
if first < 0:
    first = len(rows) + first
prev = None
busy = 0.0
for n, s, e, g in rows[first:first + count]:
    gap = (s - prev) / 1e3 if prev else 0.0
    busy += (e - s) / 1e3
    print(f"{n.split('(')[0][:60]:60s} grid {g:8d} {(e - s) / 1e3:8.2f} us  gap {gap:6.2f}")
    prev = e
print(f"busy {busy:.1f} us, span {(rows[first + count - 1][2] - rows[first][1]) / 1e3:.1f} us")
