set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_pmc_s20 PASSES="sq sq2 grbm" BENCH_ARGS="--no-cpu-baseline --no-extra --no-solve --repeats 1 --steps 20 --warmup 5" timeout -k 10 400 bash tools/pmc.sh
python3 tools/pmc_summary.py gpurun_out/r02_pmc_s20 bell_tree_kernel gpurun_out/r02_pmc_s20/summary.json 5 20
