set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_s29
mkdir -p $O
for q in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --no-ge --no-ks --no-panel > $O/bench$q.json 2> $O/bench$q.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench$q.json').read().strip().splitlines()[-1]); print(d['roofline']['kernel_avg_ms'], d['ms_per_step'], d['repeats']['median_ms_per_step'], d['repeats']['kernel_timing_block_ms_per_step'])"
done
