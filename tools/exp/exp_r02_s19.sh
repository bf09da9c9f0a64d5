set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_s19
timeout -k 10 120 python -u tools/tree_trace.py 20000 16 > gpurun_out/r02_s19/trace.txt 2>&1
