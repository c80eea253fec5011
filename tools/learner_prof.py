"""Summarise one graph-replayed learner update from a rocprofv3 kernel trace: the last N updates' kernels by name
(development tool).   python tools/learner_prof.py run_kernel_trace.csv [updates]"""
import collections, csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n_up = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 10
# updates are delimited by the replay sampler's first kernel
starts = [i for i, r in enumerate(rows) if "rp_pow" in r["Kernel_Name"]]
seg = rows[starts[-n_up]:]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seg:
    k = r["Kernel_Name"][:90]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
wall = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3 / n_up
busy = sum(v[1] for v in agg.values()) / n_up
print(f"per update: {len(seg) / n_up:.0f} kernels, wall {wall:.1f} us, busy {busy:.1f} us")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{n / n_up:6.1f}x {t / n_up:8.1f} us  {k}")
if "--seq" in sys.argv:   # the last update's kernels in launch order: start offset, duration, grid, stream
    last = rows[starts[-1]:]
    t0 = int(last[0]["Start_Timestamp"])
    for r in last:
        g = "x".join(r.get(f"Grid_Size_{a}", "?") for a in "XYZ")
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:8.1f} {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:7.1f}"
              f"  q{r.get('Queue_Id', '?'):>2} {g:>14}  {r['Kernel_Name'][:70]}")
