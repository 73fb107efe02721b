"""GPU busy time from a rocprofv3 kernel trace (run_kernel_trace.csv).

Prints the trace span, the union of kernel intervals (time with at least one kernel running),
the longest idle gaps, the time spent at each kernel concurrency level, and -- for a window
[lo, hi] ms after the first kernel -- the busy fraction per 50 ms bin, both as the sum of
kernel time (> 1 when parts overlap) and as the union.  Used to check that the interleaved
batch parts keep the device busy between their host read-backs.

    python tools/trace_busy.py <run_kernel_trace.csv> [lo_ms hi_ms]
"""
import csv
import sys


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]))
    rows.sort()
    return rows


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def bins(iv, t0, width=50.0):
    acc = {}
    for s, e in iv:
        a, b = (s - t0) / 1e6, (e - t0) / 1e6
        k = int(a // width)
        while a < b:
            nb = min(b, (k + 1) * width)
            acc[k] = acc.get(k, 0.0) + (nb - a)
            a, k = nb, k + 1
    return {k * width: v / width for k, v in sorted(acc.items())}


def main():
    rows = load(sys.argv[1])
    t0, tend = rows[0][0], max(r[1] for r in rows)
    u = union([(s, e) for s, e, _ in rows])
    busy = sum(e - s for s, e in u)
    print(f"span {(tend - t0) / 1e6:.1f} ms, {len(rows)} kernels, busy (union) {busy / 1e6:.1f} ms, "
          f"idle {(tend - t0 - busy) / 1e6:.1f} ms")
    gaps = sorted(((u[i + 1][0] - u[i][1], (u[i][1] - t0) / 1e6) for i in range(len(u) - 1)), reverse=True)
    for d, at in gaps[:10]:
        print(f"  idle gap {d / 1e6:9.3f} ms at {at:10.1f} ms")
    ev = sorted([(s, 1) for s, _, _ in rows] + [(e, -1) for _, e, _ in rows])
    lvl, last, hist = 0, ev[0][0], {}
    for t, d in ev:
        hist[lvl] = hist.get(lvl, 0) + (t - last)
        lvl, last = lvl + d, t
    print("time at each concurrency level (ms):", {k: round(v / 1e6, 1) for k, v in sorted(hist.items())})
    if len(sys.argv) > 3:
        lo, hi = float(sys.argv[2]), float(sys.argv[3])
        sel = [(s, e) for s, e, _ in rows if lo <= (s - t0) / 1e6 <= hi]
        print("kernel-time / wall per 50 ms:", " ".join(f"{k:.0f}:{v:.2f}" for k, v in bins(sel, t0).items()))
        print("union busy / wall per 50 ms:  ", " ".join(f"{k:.0f}:{v:.2f}" for k, v in bins(union(sel), t0).items()))


if __name__ == "__main__":
    main()
