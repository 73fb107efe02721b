"""Summarise rocprofv3 outputs (kernel stats CSV + --pmc counter CSVs) into profiles/.

usage: python tools/profile_summary.py <stats_dir> [<pmc_dir> ...] > profiles/<round>_summary.txt
FETCH_SIZE / WRITE_SIZE are reported in KB per dispatch by rocprofv3; on gfx950 FETCH_SIZE
counts half the bytes of wide (16 B/lane) coalesced reads (MI355X_MICROARCH.md, HBM), so the
corrected HBM read bytes are 2 x FETCH_SIZE for the streaming GEMM/quantiser kernels.
"""
import collections
import csv
import glob
import os
import sys


def stats(d):
    f = glob.glob(os.path.join(d, "*kernel_stats.csv"))[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# kernel stats: {f}  (total GPU kernel time {tot / 1e6:.2f} ms)")
    print(f"{'total_ms':>10} {'pct':>6} {'calls':>6} {'avg_us':>10}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        print(f"{float(r['TotalDurationNs']) / 1e6:10.2f} {float(r['Percentage']):6.2f} {r['Calls']:>6} "
              f"{float(r['AverageNs']) / 1e3:10.1f}  {r['Name'][:110]}")


def by_grid(d, pattern="gemm_x3v_kernel"):
    """Launches of the split-fp16 product kernels grouped by (instantiation, grid): the filter,
    Rayleigh-Ritz and U^T Y products share one grid (M = p rows, N = k), the Gram has its own."""
    fs = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    if not fs:
        return
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        if pattern in r["Kernel_Name"]:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[(r["Kernel_Name"], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))].append(dur)
    print(f"# {pattern} launches by grid: {fs[0]}")
    print(f"{'calls':>6} {'avg_us':>10} {'workgroups':>10}  kernel")
    for (k, g), v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        print(f"{len(v):>6} {sum(v) / len(v):10.1f} {g:>10}  {k[:80]}")


def pmc(d):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(list)
    for r in rows:
        wg = int(r.get("Grid_Size", 0) or 0) // max(1, int(r.get("Workgroup_Size", 1) or 1))
        agg[(r["Kernel_Name"], r["Counter_Name"], wg)].append(float(r["Counter_Value"]))
    print(f"# PMC: {f}")
    print(f"{'counter':>12} {'dispatches':>10} {'avg_KB':>14} {'workgroups':>10}  kernel")
    for (k, c, wg), v in sorted(agg.items(), key=lambda x: -sum(x[1]))[:20]:
        print(f"{c:>12} {len(v):>10} {sum(v) / len(v):14.1f} {wg:>10}  {k[:100]}")


if __name__ == "__main__":
    stats(sys.argv[1])
    print()
    by_grid(sys.argv[1])
    for d in sys.argv[2:]:
        print()
        pmc(d)
