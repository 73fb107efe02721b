set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r06q/kt gpurun_out/r06q/kt1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r06q/kt -o run --output-format csv -- python3 bench.py > gpurun_out/r06q/bench_default_ktrace.log 2>&1
python3 tools/ktrace_summary.py gpurun_out/r06q/kt_tmp 2>/dev/null || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06q/kt1 -o run --output-format csv -- python3 bench.py --streams 1 --steps 1 --warmup 1 --no-parity --no-cpu-baseline --no-api-path > gpurun_out/r06q/kt1.log 2>&1
