# per-(kernel, grid) breakdown of bench.py runs: rocprofv3 --kernel-trace
# usage: bash tools/ktrace.sh <tag> <bench args...>
set -e
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out/kt_$tag
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/kt_$tag/t -o run --output-format csv -- python3 bench.py "$@" > gpurun_out/kt_$tag/s.log 2>&1
python3 tools/ktrace_summary.py gpurun_out/kt_$tag > gpurun_out/kt_$tag/summary.txt
cat gpurun_out/kt_$tag/summary.txt
