set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/kt_single
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_single/t -o run --output-format csv -- python3 tools/bench_single.py 5 > gpurun_out/kt_single/s.log 2>&1
python3 tools/ktrace_summary.py gpurun_out/kt_single > gpurun_out/kt_single/summary.txt
f=$(ls gpurun_out/kt_single/t/*/run_kernel_trace.csv 2>/dev/null || find gpurun_out/kt_single/t -name run_kernel_trace.csv | head -1)
python3 tools/trace_busy.py $(find gpurun_out/kt_single/t -name run_kernel_trace.csv | head -1) > gpurun_out/kt_single/busy.txt
rm -rf gpurun_out/kt_single/t
