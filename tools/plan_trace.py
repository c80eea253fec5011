"""Per-kernel breakdown of one plan() from a rocprofv3 kernel trace (development tool).

    python tools/plan_trace.py run_kernel_trace.csv [plans_back]
A plan is delimited by its cem_kernel launches (iterations); the last complete plan is summarised."""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cem = [i for i, r in enumerate(rows) if "cem_kernel" in r["Kernel_Name"]]
# iterations per plan: count cem launches between encode launches
enc = [i for i, r in enumerate(rows) if "encode_kernel" in r["Kernel_Name"]]
a = enc[-1 - back]
b = [i for i in cem if i > a]
iters = len([i for i in cem if a < i < enc[-back]]) if back > 0 else len(b)
end = [i for i in cem if a < i][iters - 1] + 1
seg = rows[a:end]


def nm(r):
    m = re.search(r"::(\w+)(<[^>]*>)?", r["Kernel_Name"])
    return (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]


t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"plan: {len(seg)} kernels, {iters} iterations, wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
tot = collections.defaultdict(list)
for r in seg:
    k = (nm(r), int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))
    tot[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(tot.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k[0]:48s} grid {k[1]:4d}x{k[2]:2d}x{k[3]}  n={len(v):3d}  avg {sum(v) / len(v):7.2f} us  total {sum(v):8.1f} us")
