"""One graph-replayed learner update's kernel sequence from a rocprofv3 kernel trace (development tool).
    python tools/learner_seq.py run_kernel_trace.csv > seq.txt"""
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "rp_pow" in r["Kernel_Name"]]
seg = rows[starts[-2]:starts[-1]]
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.2f}  {r['Kernel_Name'][:150]}")
