"""Per-launch HBM traffic of one kernel from rocprofv3 PMC passes (development/profiling tool).

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV KERNEL_SUBSTR GRID_SIZE KEY [FLOPS_PER_LAUNCH]

FETCH_SIZE / WRITE_SIZE are collected in separate passes (TCC slots, MI355X_MICROARCH.md §rocprofv3 PMC
slots). Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports half the bytes of wide (16 B per
lane) coalesced reads -- every load of the linear kernels is one -- so bytes = 2 * FETCH_SIZE(KB) * 1024 +
WRITE_SIZE(KB) * 1024. The result is merged into profiles/pmc_traffic.json under KEY.
"""
import csv
import json
import os
import statistics
import sys


def per_dispatch(path, counter, kname, grid):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or kname not in r["Kernel_Name"] or r["Grid_Size"] != grid:
            continue
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fetch_csv, write_csv, kname, grid, key = sys.argv[1:6]
    fetch = per_dispatch(fetch_csv, "FETCH_SIZE", kname, grid)
    write = per_dispatch(write_csv, "WRITE_SIZE", kname, grid)
    if not fetch or not write:
        raise SystemExit(f"no dispatches of {kname} grid {grid}: {len(fetch)} / {len(write)}")
    f_kb, w_kb = statistics.median(fetch), statistics.median(write)
    hbm = 2 * f_kb * 1024 + w_kb * 1024
    out_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                            "pmc_traffic.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {}
    data[key] = {"kernel": kname, "grid_size": int(grid), "dispatches": len(fetch),
                 "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
                 "hbm_bytes_per_launch": hbm,
                 "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bytes = 2*FETCH + WRITE"}
    json.dump(data, open(out_path, "w"), indent=1)
    print(json.dumps(data[key]))


if __name__ == "__main__":
    main()
