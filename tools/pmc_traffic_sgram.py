"""Per-dispatch HBM traffic of the sparse-code Gram kernels (sgram.py) and the LR step's
residual pass from two rocprofv3 --pmc passes of bench.py (FETCH_SIZE, WRITE_SIZE), against
their algorithmic bytes per B-matrix launch (m <= n, k = m):
  sgram_spmm      W (2mn) + 2-bit codes (mn/4) read, P (4k^2) written (+ the ELL, ~4 nnz)
  sgram_combine   A's upper triangle (2k^2) + P (4k^2) read, G's split halves (4k^2) written
  residual_split  W + codes read, Y^T's split halves (4mn) written (the run's first call writes
                  W's halves for A instead: same bytes without the codes)
usage: python tools/pmc_traffic_sgram.py <fetch_dir> <write_dir> <batch> <m> <n>
hbm = 2 * FETCH_SIZE + WRITE_SIZE (KB * 1024), gfx950 (MI355X_MICROARCH.md, HBM)."""
import csv, glob, json, os, statistics, sys

fetch_dir, write_dir = sys.argv[1], sys.argv[2]
B, m, n = (int(x) for x in sys.argv[3:6])


def vals(d, name):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    out = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == name:
            out.setdefault(r["Kernel_Name"].split("(")[0], []).append(float(r["Counter_Value"]))
    return out


fe, wr = vals(fetch_dir, "FETCH_SIZE"), vals(write_dir, "WRITE_SIZE")
k = m
alg = {"sgram_spmm": ("P = (W - s/2 c) c^T over the ELL codes", B * (2 * m * n + m * n // 4 + 4 * k * k)),
       "sgram_combine": ("G = A - s (P + P^T) -> split halves", B * 10 * k * k),
       "residual_split": ("LR-step residual: Y^T halves + ||Y||^2", B * (2 * m * n + m * n // 4 + 4 * m * n))}
res = {}
for name in sorted(fe):
    tag = next((t for t in alg if t in name), None)
    if tag is None or name not in wr:
        continue
    fk, wk = statistics.mean(fe[name]), statistics.mean(wr[name])
    hbm = (2 * fk + wk) * 1024
    res[tag] = {"kernel": name, "what": alg[tag][0], "dispatches": len(fe[name]), "FETCH_SIZE_KB_avg": fk,
                "WRITE_SIZE_KB_avg": wk, "hbm_bytes_per_dispatch": hbm,
                "algorithmic_bytes_per_dispatch": alg[tag][1], "ratio": hbm / alg[tag][1]}
print(json.dumps({"config": {"batch": B, "m": m, "n": n}, "kernels": res,
                  "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KB*1024), gfx950 (MI355X_MICROARCH.md HBM)"},
                 indent=1))
