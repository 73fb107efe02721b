"""Summary of tools/pmc_mfma.sh: per (kernel, workgroups) the mean of every counter per
dispatch and the derived figures -- MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over the
CUs' cycles, GRBM_GUI_ACTIVE / 8 XCDs being one CU's clock count), effective clock, and the
wave-cycle split (SQ_* in quad-cycles: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES).
Writes OUT/summary.json and prints a table."""
import collections
import csv
import glob
import json
import os
import sys

CUS = 256


def load(out):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            wg = int(r.get("Grid_Size", 0) or 0) // max(1, int(r.get("Workgroup_Size", 1) or 1))
            key = (r["Kernel_Name"].split("(")[0][:90], wg)
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return agg, dur


def main(out):
    agg, dur = load(out)
    res = {}
    for key, cs in sorted(agg.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = {"kernel": key[0], "workgroups": key[1], "dispatches": max(len(v) for v in cs.values()),
             "counters": m}
        if dur.get(key):
            d["profiled_ms"] = sorted(dur[key])[len(dur[key]) // 2]
        gui = m.get("GRBM_GUI_ACTIVE")
        if gui:
            cyc = gui / 8.0  # one XCD's busy cycles = the dispatch's cycles at the shader clock
            if d.get("profiled_ms"):
                d["effective_clock_ghz"] = cyc / (d["profiled_ms"] * 1e6)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                # SQ_VALU_MFMA_BUSY_CYCLES: summed over the CUs (4 SIMDs each, cycles of MFMA busy)
                d["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (CUS * 4 * cyc)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
                if c in m:
                    d[c.lower() + "_frac_of_wave_cycles"] = m[c] / wc
        res[f"{key[0]} [{key[1]} wg]"] = d
    json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
    for k, d in res.items():
        extra = " ".join(f"{a}={d[a]:.3f}" for a in ("mfma_busy_frac", "effective_clock_ghz") if a in d)
        print(f"{k[:100]:100s} n={d['dispatches']:4d} {extra}")
        for c, v in sorted(d["counters"].items()):
            print(f"      {c:30s} {v:16.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
