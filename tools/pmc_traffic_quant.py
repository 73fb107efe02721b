"""Per-dispatch HBM traffic of the quantise kernels from two rocprofv3 --pmc passes of
bench.py (FETCH_SIZE, WRITE_SIZE), against their algorithmic bytes.

usage: python tools/pmc_traffic_quant.py <fetch_dir> <write_dir> <batch> <m> <n> <bits>
gfx950 FETCH_SIZE counts half the bytes of 16 B/lane streaming reads (MI355X_MICROARCH.md,
HBM), so hbm = 2 * FETCH_SIZE + WRITE_SIZE (KB * 1024)."""
import csv, glob, json, os, statistics, sys

fetch_dir, write_dir = sys.argv[1], sys.argv[2]
B, m, n, bits = (int(x) for x in sys.argv[3:7])


def vals(d, name):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    out = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != name:
            continue
        k = r["Kernel_Name"].split("(")[0]
        out.setdefault(k, []).append(float(r["Counter_Value"]))
    return out


fe, wr = vals(fetch_dir, "FETCH_SIZE"), vals(write_dir, "WRITE_SIZE")
w_bytes, code_bytes = 2 * m * n, m * n * bits // 8
res = {}
for k in sorted(fe):
    if k not in wr or not any(t in k for t in ("quant_w_stream", "q_update_p", "q_update_v")):
        continue
    fk, wk = statistics.mean(fe[k]), statistics.mean(wr[k])
    if "quant_w_stream" in k:
        alg, what = B * (w_bytes + code_bytes), "first Q step (max|W| known): W read + packed codes written"
    elif "<0" in k:
        alg, what = B * w_bytes, "Q update pass 0 (absmax of W - L R): W read"
    else:
        alg, what = B * (w_bytes + code_bytes), "Q update pass 1 (quantise W - L R): W read + packed codes written"
    res[k] = {"what": what, "dispatches": len(fe[k]), "FETCH_SIZE_KB_avg": fk, "WRITE_SIZE_KB_avg": wk,
              "hbm_bytes_per_dispatch": (2 * fk + wk) * 1024, "algorithmic_bytes_per_dispatch": alg}
print(json.dumps({"config": {"batch": B, "m": m, "n": n, "bits": bits}, "kernels": res,
                  "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KB*1024), gfx950 (MI355X_MICROARCH.md HBM)",
                  "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) "
                            f"--kernel-include-regex 'quant_w_stream|q_update_p|q_update_v' -- python3 bench.py --batch {B} "
                            f"--steps 1 --warmup 0 --no-parity --no-cpu-baseline --no-api-path"}, indent=1))
