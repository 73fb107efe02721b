"""Per-launch HBM traffic of the filter GEMM from two rocprofv3 --pmc passes of bench.py.

usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <batch> <p> <k> > profiles/pmc_traffic.json
Filter launches are the gemm_x3 dispatches whose grid is the filter's (M = p rows of X^T,
N = k columns); gfx950 FETCH_SIZE counts half the bytes of 16 B/lane streaming reads
(MI355X_MICROARCH.md, HBM), so hbm = 2 * FETCH_SIZE + WRITE_SIZE (KB * 1024)."""
import csv, glob, json, os, statistics, sys

fetch_dir, write_dir, B, p, k = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
XW_BM, XW_BN, XW_THREADS = 192, 384, 768
grid = ((k + XW_BN - 1) // XW_BN) * ((p + XW_BM - 1) // XW_BM) * B * XW_THREADS


def vals(d, name, single):
    """Dispatches of the filter grid; single: the one-product (hi x hi) instantiation
    gemm_x3v_kernel<1> of the cheap outer iterations, else the split-fp16 <0> one."""
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    tag = "gemm_x3v_kernel<1>" if single else "gemm_x3v_kernel<0>"
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if tag in r["Kernel_Name"] and int(r["Grid_Size"]) == grid and r["Counter_Name"] == name]


fe, wr = vals(fetch_dir, "FETCH_SIZE", False), vals(write_dir, "WRITE_SIZE", False)
fk, wk = statistics.mean(fe), statistics.mean(wr)
alg = B * (4.0 * k * k + 20.0 * p * k)
fe1, wr1 = vals(fetch_dir, "FETCH_SIZE", True), vals(write_dir, "WRITE_SIZE", True)
single = None
if fe1 and wr1:
    f1, w1 = statistics.mean(fe1), statistics.mean(wr1)
    # hi halves only: G hi 2k^2 + X^T hi 2pk, P and D 8pk in, C 4pk + halves 4pk out
    single = {"kernel": "gemm_x3v_kernel<1> (one fp16 product, cheap outer iterations)", "dispatches": len(fe1),
              "FETCH_SIZE_KB_avg": f1, "WRITE_SIZE_KB_avg": w1, "hbm_bytes_per_launch": (2 * f1 + w1) * 1024,
              "algorithmic_bytes_per_launch": B * (2.0 * k * k + 18.0 * p * k)}
out = {
    "kernel": "gemm_x3v_kernel<0> (split-fp16 G X, Chebyshev filter)",
    "config": {"batch": B, "p": p, "k": k},
    "dispatches": len(fe),
    "FETCH_SIZE_KB_avg": fk, "WRITE_SIZE_KB_avg": wk,
    "hbm_bytes_per_launch": (2 * fk + wk) * 1024,
    "algorithmic_bytes_per_launch": alg,
    "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KB*1024); gfx950 FETCH_SIZE counts half of 16 B/lane "
                  "coalesced reads (MI355X_MICROARCH.md HBM); includes the 13 Rayleigh-Ritz G X launches "
                  "of the same grid (no recurrence operands); the single-product launches are reported apart",
    "single_product_launches": single,
    "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-include-regex gemm_x3 "
              f"-- python3 bench.py --batch {B} --steps 1 --warmup 0 --no-parity",
}
print(json.dumps(out, indent=1))
