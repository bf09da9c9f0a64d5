set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02_s21
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/r02_s21/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra --repeats 1 --steps 20 --warmup 5 > gpurun_out/r02_s21/bench.log 2>&1
tail -1 gpurun_out/r02_s21/bench.log | cut -c1-200
find gpurun_out/r02_s21/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160 | head -20
