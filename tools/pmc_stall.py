"""Median per-dispatch counter values of one kernel from rocprofv3 --pmc CSVs (development/profiling tool).

    python tools/pmc_stall.py KERNEL_SUBSTR GRID_SIZE CSV [CSV ...]
"""
import collections
import csv
import statistics
import sys


def main():
    kname, grid = sys.argv[1:3]
    out = {}
    for path in sys.argv[3:]:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            if kname not in r["Kernel_Name"] or r["Grid_Size"] != grid:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names = sorted({n for v in per.values() for n in v})
        for n in names:
            out[n] = statistics.median(v[n] for v in per.values())
    for n, v in out.items():
        print(f"{n:32s} {v:16.0f}")
    w = out.get("SQ_WAVE_CYCLES")
    if w:
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS"):
            if n in out:
                print(f"{n} / SQ_WAVE_CYCLES = {out[n] / w:.3f}")


if __name__ == "__main__":
    main()
