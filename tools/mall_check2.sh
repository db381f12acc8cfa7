cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1 || { tail -30 gpurun_out/pytest_parity.log; exit 1; }
tail -1 gpurun_out/pytest_parity.log
timeout -k 10 200 python bench.py --no-cpu-baseline --warmup 100 --nx 6144 --ny 6144 > gpurun_out/mall_6144_default2.log 2>&1 || exit 1
echo DONE
