"""Group a rocprofv3 kernel trace by (kernel, grid, workgroup) and print time shares."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
f = (glob.glob(f"{d}/t/**/run_kernel_trace.csv", recursive=True) or glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    key = (r["Kernel_Name"][:70], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""),
           r.get("Grid_Size_Z", ""), r.get("Workgroup_Size_X", r.get("Workgroup_Size", "")))
    a = agg[key]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
tot = sum(v[1] for v in agg.values())
print(f"total {tot:.1f} ms over {len(rows)} launches")
for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{100 * ms / tot:6.2f}% {ms:9.2f} ms {n:5d} x {ms / n:8.3f} ms  grid {k[1]}x{k[2]}x{k[3]} wg {k[4]}  {k[0]}")
