set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/ge_timing.py
