set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_g1_tests.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r04_g1_bench.out 2> gpurun_out/r04_g1_bench.err
rc=$?
tail -3 gpurun_out/r04_g1_tests.log; tail -c 600 gpurun_out/r04_g1_bench.out
exit $rc
