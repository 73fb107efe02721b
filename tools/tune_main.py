"""GPU tool: bench.py --workload main (main.py's layer set, per-layer real Hessians, batched and
as the one-call-per-layer loop) under solver settings given as NAME=VALUE module overrides of
ee274_convexcaldera_llm_quantization_amd.solver (e.g. SEGMENTS_MAX=4), one JSON line each.
    python tools/tune_main.py SEGMENTS_MAX=1 SEGMENTS_MAX=4 ...
    python tools/tune_main.py --workload cfg2 SEGMENTS_MAX=1 ...   (any other bench workload, its
                                                                   timed region without parity)"""
import argparse
import contextlib
import io
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ee274_convexcaldera_llm_quantization_amd")]

import bench  # noqa: E402
from ee274_convexcaldera_llm_quantization_amd import solver  # noqa: E402


def main():
    argv = sys.argv[1:]
    wl = "main"
    if argv[:1] == ["--workload"]:
        wl, argv = argv[1], argv[2:]
    for spec in argv or [""]:
        saved = {}
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            saved[k] = getattr(solver, k)
            setattr(solver, k, type(saved[k])(eval(v)))
        buf = io.StringIO()
        if wl == "main":
            with contextlib.redirect_stdout(buf):
                bench.run_main(argparse.Namespace(steps=2, warmup=1))
            d = json.loads(buf.getvalue().strip().splitlines()[-1])
            print(json.dumps({"spec": spec, "matrices_per_s": round(d["value"], 1),
                              "b1_ms_per_layer": round(d["b1_loop"]["ms_per_layer"], 1),
                              "batched_vs_b1": d["batched_vs_b1"]}), flush=True)
        else:
            sys.argv = ["bench.py", "--workload", wl, "--no-cpu-baseline", "--no-parity", "--no-api-path"]
            with contextlib.redirect_stdout(buf):
                bench.main()
            d = json.loads(buf.getvalue().strip().splitlines()[-1])
            print(json.dumps({"spec": spec, "workload": wl, "value": round(d["value"], 1),
                              "ms_per_step": round(d["ms_per_step"], 2)}), flush=True)
        for k, v in saved.items():
            setattr(solver, k, v)


if __name__ == "__main__":
    main()
