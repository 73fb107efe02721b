"""Per-launch HBM traffic of the filter GEMM from two rocprofv3 --pmc passes of bench.py.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <batch> <p> <k> > profiles/pmc_traffic.json
Filter launches are the gemm_x3 dispatches whose grid is the filter's (M = p rows of X^T,
N = k columns); gfx950 FETCH_SIZE counts half the bytes of 16 B/lane streaming reads
(MI355X_MICROARCH.md, HBM), so hbm = 2 * FETCH_SIZE + WRITE_SIZE (KB * 1024)."""
import csv, glob, json, os, statistics, sys

fetch_dir, write_dir, B, p, k = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
XW_BM, XW_BN, XW_THREADS = 192, 384, 768
grid = ((k + XW_BN - 1) // XW_BN) * ((p + XW_BM - 1) // XW_BM) * B * XW_THREADS


def vals(d, name):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if "gemm_x3" in r["Kernel_Name"] and int(r["Grid_Size"]) == grid and r["Counter_Name"] == name]


fe, wr = vals(fetch_dir, "FETCH_SIZE"), vals(write_dir, "WRITE_SIZE")
fk, wk = statistics.mean(fe), statistics.mean(wr)
alg = B * (4.0 * k * k + 20.0 * p * k)
out = {
    "kernel": "gemm_x3_kernel (split-fp16 G X, Chebyshev filter)",
    "config": {"batch": B, "p": p, "k": k},
    "dispatches": len(fe),
    "FETCH_SIZE_KB_avg": fk, "WRITE_SIZE_KB_avg": wk,
    "hbm_bytes_per_launch": (2 * fk + wk) * 1024,
    "algorithmic_bytes_per_launch": alg,
    "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KB*1024); gfx950 FETCH_SIZE counts half of 16 B/lane "
                  "coalesced reads (MI355X_MICROARCH.md HBM); includes the 13 Rayleigh-Ritz G X launches "
                  "of the same grid (no recurrence operands)",
    "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-include-regex gemm_x3 "
              f"-- python3 bench.py --batch {B} --steps 1 --warmup 0 --no-parity",
}
print(json.dumps(out, indent=1))
