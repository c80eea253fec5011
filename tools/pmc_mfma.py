"""MFMA utilisation of one kernel from a rocprofv3 PMC pass (development/profiling tool).

    python tools/pmc_mfma.py COUNTER_CSV KERNEL_SUBSTR GRID_SIZE KEY

Pass: rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES (tools/gpu41.sh).
utilisation = SQ_VALU_MFMA_BUSY_CYCLES (summed over the 1024 SIMDs) / (GRBM_GUI_ACTIVE / 8 x 1024), i.e. the
rocprofv3 'MfmaUtil' derived metric (reduce(GRBM_GUI_ACTIVE, max) = the per-XCD value = the 8-XCD sum / 8);
the effective clock is GRBM_GUI_ACTIVE / 8 / dispatch wall time (MI355X_MICROARCH.md 'DVFS give-back').
The result is merged into profiles/pmc_mfma.json under KEY.
"""
import collections
import csv
import json
import os
import statistics
import sys

SIMDS = 1024   # 256 CUs x 4


def main():
    path, kname, grid, key = sys.argv[1:5]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    wall = {}
    for r in csv.DictReader(open(path)):
        if kname not in r["Kernel_Name"] or r["Grid_Size"] != grid:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        wall[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    if not per:
        raise SystemExit(f"no dispatches of {kname} grid {grid}")
    busy = statistics.median(v["SQ_VALU_MFMA_BUSY_CYCLES"] for v in per.values())
    grbm = statistics.median(v["GRBM_GUI_ACTIVE"] for v in per.values())
    ns = statistics.median(wall.values())
    out = {"kernel": kname, "grid_size": int(grid), "dispatches": len(per),
           "sq_valu_mfma_busy_cycles_median": busy, "grbm_gui_active_median": grbm,
           "mfma_util": round(busy / (grbm / 8 * SIMDS), 4),
           "clock_ghz": round(grbm / 8 / ns, 3), "dispatch_us_median_profiled": ns / 1e3,
           "source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES; "
                     "util = MFMA busy SIMD-cycles / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)"}
    op = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_mfma.json")
    data = json.load(open(op)) if os.path.exists(op) else {}
    data[key] = out
    json.dump(data, open(op, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
