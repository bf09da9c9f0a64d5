set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r02_pmc_s24q PASSES="sq sq2 grbm" BENCH_ARGS="--no-cpu-baseline --no-extra --no-solve --no-ge --no-ks --no-panel --repeats 1 --steps 20 --warmup 5 --variant 80" timeout -k 10 400 bash tools/pmc.sh
python3 tools/pmc_summary.py gpurun_out/r02_pmc_s24q bell_quad_kernel gpurun_out/r02_pmc_s24q/summary.json 5 20 | tail -16
OUT=gpurun_out/r02_pmc_s24t PASSES="sq sq2 grbm" BENCH_ARGS="--no-cpu-baseline --no-extra --no-solve --no-ge --no-ks --no-panel --repeats 1 --steps 20 --warmup 5" timeout -k 10 400 bash tools/pmc.sh
python3 tools/pmc_summary.py gpurun_out/r02_pmc_s24t bell_tree_kernel gpurun_out/r02_pmc_s24t/summary.json 5 20 | tail -16
