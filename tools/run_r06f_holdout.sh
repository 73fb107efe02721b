set -e
mkdir -p gpurun_out
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-api-path"
timeout -k 10 240 $B > gpurun_out/r06f_default.json 2> gpurun_out/r06f_default.err
timeout -k 10 240 $B --deg-cold 6,12,10 > gpurun_out/r06f_cold61210.json 2> gpurun_out/r06f_cold.err
timeout -k 10 240 $B --solver-tol-steps 3e-6,3e-6,3e-6,3e-6,3e-6 > gpurun_out/r06f_tol3e6.json 2> gpurun_out/r06f_tol3.err
timeout -k 10 240 $B --solver-tol-steps 5e-6,5e-6,5e-6,5e-6,5e-6 > gpurun_out/r06f_tol5e6.json 2> gpurun_out/r06f_tol5.err
