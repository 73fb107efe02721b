# GPU box: kernel stats of one bench step (batch $1) -> gpurun_out/prof_$2
set -eo pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B=${1:-256}; TAG=${2:-tmp}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- \
    python3 bench.py --batch $B --steps 1 --warmup 1 --no-parity > $OUT/stats.log 2>&1
python3 tools/profile_summary.py $OUT/stats > $OUT/summary.txt
head -25 $OUT/summary.txt
