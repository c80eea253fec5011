"""Summarise a rocprofv3 kernel-trace CSV: per (kernel, grid, block) average duration and share."""
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ncalls = int(sys.argv[2]) if len(sys.argv) > 2 else 1
d = collections.defaultdict(list)
for x in rows:
    k = (x['Kernel_Name'][:28], int(x['Grid_Size_X']) // int(x['Workgroup_Size_X']), x['Grid_Size_Y'], x['Grid_Size_Z'], x['Workgroup_Size_X'])
    d[k].append(int(x['End_Timestamp']) - int(x['Start_Timestamp']))
tot = sum(sum(v) for v in d.values())
print(f"total kernel time {tot/1e6:.3f} ms over {ncalls} calls = {tot/1e3/ncalls:.1f} us/call")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:25]:
    print(f"{str(k):70s} n={len(v):5d} avg={sum(v)/len(v)/1e3:8.2f}us  per_call={sum(v)/1e3/ncalls:8.1f}us  {100*sum(v)/tot:5.1f}%")
