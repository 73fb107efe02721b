"""Per-(kernel, grid) HBM bytes per dispatch from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE in separate runs of the same command), gfx950-corrected: hbm = 2 FETCH + WRITE
(KB x 1024; MI355X_MICROARCH.md, HBM).  usage: python tools/pmc_sum.py <fetch_dir> <write_dir> [name substrings]"""
import collections
import csv
import glob
import json
import os
import sys

fetch_dir, write_dir = sys.argv[1], sys.argv[2]
keys = sys.argv[3:]


def vals(d, name):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != name:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if keys and not any(s in k for s in keys):
            continue
        grid = r.get("Grid_Size", r.get("Grid_Size_X", ""))
        out[(k, grid)].append(float(r["Counter_Value"]))
    return out


fe, wr = vals(fetch_dir, "FETCH_SIZE"), vals(write_dir, "WRITE_SIZE")
res = {}
for k in sorted(fe):
    if k not in wr:
        continue
    f, w = sum(fe[k]) / len(fe[k]), sum(wr[k]) / len(wr[k])
    res[f"{k[0]} grid {k[1]}"] = {"dispatches": len(fe[k]), "fetch_bytes": 2 * f * 1024, "write_bytes": w * 1024,
                                  "hbm_bytes_per_dispatch": (2 * f + w) * 1024}
print(json.dumps({"kernels": res, "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KB*1024), gfx950"}, indent=1))
