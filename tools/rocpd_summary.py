"""Per-kernel summary of a rocprofv3 rocpd database (development tool):
    python tools/rocpd_summary.py run_results.db [N] [--grid]
--grid: one row per (kernel, grid x * y * z work-items) instead of per kernel."""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 30
by_grid = "--grid" in sys.argv
q = ("select s.kernel_name, d.start, d.end, d.grid_size_x * d.grid_size_y * d.grid_size_z from rocpd_kernel_dispatch d "
     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
agg = collections.defaultdict(list)
for n, s, e, g in c.execute(q):
    k = n.split("(")[0]
    agg[f"{k[:76]} grid {g}" if by_grid else k].append((e - s) / 1e3)
tot = sum(sum(v) for v in agg.values())
print(f"{'kernel':90s} {'n':>6s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{k[:90]:90s} {len(v):6d} {sum(v) / len(v):9.2f} {sum(v) / 1e3:9.3f} {100 * sum(v) / tot:6.2f}")
