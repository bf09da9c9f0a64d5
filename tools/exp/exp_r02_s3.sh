export TMPDIR=/tmp
mkdir -p gpurun_out/r02_s3
timeout -k 10 300 python -u -m pytest tests/test_vfi_gpu.py tests/test_spec_solve_gpu.py tests/test_labor_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_s3/pytest.log 2>&1 || { tail -30 gpurun_out/r02_s3/pytest.log; exit 1; }
tail -3 gpurun_out/r02_s3/pytest.log
TAG=r02_s3v VARIANTS="0 32" bash tools/variant_sweep.sh || exit 1
for v in 0 32; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/r02_s3/tr$v -o run -- python3 $PWD/bench.py --no-cpu-baseline --no-ge --no-ks --no-panel --steps 20 --warmup 5 --variant $v > gpurun_out/r02_s3/tr$v.log 2>&1 || exit 1
python3 tools/sweep_times.py gpurun_out/r02_s3/tr$v bell_tree_kernel 0 25
python3 tools/sweep_times.py gpurun_out/r02_s3/tr$v bell_tree_kernel 28
done
