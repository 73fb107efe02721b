"""Summarise rocprofv3 --pmc counter CSVs: per (kernel, grid, counter) the mean value."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    fs = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not fs:
        print(f"# {d}: no counter file")
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        wg = int(r.get("Grid_Size", 0) or 0) // max(1, int(r.get("Workgroup_Size", 1) or 1))
        agg[(r["Kernel_Name"][:70], wg, r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(f"# {fs[0]}")
    for (k, wg, c), v in sorted(agg.items()):
        print(f"{c:28s} {len(v):4d} {sum(v) / len(v):18.1f} {wg:8d}  {k}")
