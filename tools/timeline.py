"""Timeline of the LAST step of a rocprofv3 kernel trace whose steps are separated by idle
gaps (tools/bench_share.py): wall time, GPU-busy time (union of kernel intervals), idle gaps
(host-bound stretches), the kernels by summed time, and the concurrency profile.

  python tools/timeline.py <trace dir> [gap_ms=20]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
gap_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in rows]
# split into steps at idle gaps
segs, cur, end = [], [], None
for s, e, r in iv:
    if end is not None and s - end > gap_ms * 1e6:
        segs.append(cur)
        cur = []
    cur.append((s, e, r))
    end = e if end is None else max(end, e)
segs.append(cur)
seg = segs[-1]
t0 = seg[0][0]
t1 = max(e for _, e, _ in seg)
wall = (t1 - t0) / 1e6
busy, idle, gaps = 0.0, 0.0, []
ce = t0
for s, e, _ in seg:
    if s > ce:
        g = (s - ce) / 1e6
        idle += g
        gaps.append((g, (ce - t0) / 1e6))
    if e > ce:
        busy += (e - max(s, ce)) / 1e6
        ce = e
print(f"{len(segs)} segments; last: {len(seg)} launches, wall {wall:.2f} ms, GPU busy {busy:.2f} ms, "
      f"idle {idle:.2f} ms in {len(gaps)} gaps")
big = sorted(gaps, reverse=True)[:15]
print("largest idle gaps (ms @ offset ms):", ", ".join(f"{g:.2f}@{o:.1f}" for g, o in big))
hist = collections.Counter()
for g, _ in gaps:
    hist["<0.02" if g < 0.02 else "<0.1" if g < 0.1 else "<0.5" if g < 0.5 else "<2" if g < 2 else ">=2"] += 1
print("gap histogram:", dict(hist))
agg = collections.defaultdict(lambda: [0, 0.0])
for s, e, r in seg:
    k = (r["Kernel_Name"][:80], r.get("Grid_Size_X", r.get("Grid_Size", "")))
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e6
tot = sum(v[1] for v in agg.values())
print(f"kernel time summed {tot:.2f} ms (concurrency {tot / max(busy, 1e-9):.2f}x while busy)")
for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{ms:8.2f} ms {n:5d} x {ms / n:7.3f}  grid {k[1]:>9}  {k[0]}")
# concurrency: time with 0, 1, 2, 3+ kernels running
ev = sorted([(s, 1) for s, _, _ in seg] + [(e, -1) for _, e, _ in seg])
conc = collections.Counter()
c, last = 0, t0
for t, dlt in ev:
    conc[min(c, 4)] += (t - last) / 1e6
    c += dlt
    last = t
print("time by kernels in flight:", {k: round(v, 2) for k, v in sorted(conc.items())})
# per stream: summed kernel time, first/last timestamps, and top kernels
ps = collections.defaultdict(lambda: [0.0, None, None, collections.Counter(), 0])
for s, e, r in seg:
    key = r.get("Stream_Id", r.get("Queue_Id"))
    p = ps[key]
    p[0] += (e - s) / 1e6
    p[1] = s if p[1] is None else min(p[1], s)
    p[2] = e if p[2] is None else max(p[2], e)
    p[3][r["Kernel_Name"][:60]] += (e - s) / 1e6
    p[4] += 1
for key, (ms, a, b, c, n) in sorted(ps.items(), key=lambda kv: -kv[1][0]):
    print(f"stream {key}: {n} launches, kernels {ms:.2f} ms, span {(a - t0) / 1e6:.1f} .. {(b - t0) / 1e6:.1f} ms; "
          + "; ".join(f"{k[:40]} {v:.1f}" for k, v in c.most_common(5)))
