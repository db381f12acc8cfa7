# GPU: tests, then the default geometry choice on grids around the Infinity
# Cache size (one bench process per setting).
cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --warmup 100 "$@" || exit 1; }
run --nx 8192 --ny 4096 > gpurun_out/mall_8192x4096_default.log 2>&1
CFD_TEMPORAL=4 run --nx 8192 --ny 4096 > gpurun_out/mall_8192x4096_t4.log 2>&1
run --nx 8192 --ny 8192 > gpurun_out/mall_8192x8192_default.log 2>&1
run --nx 6144 --ny 6144 > gpurun_out/mall_6144_default.log 2>&1
CFD_TEMPORAL=4 run --nx 6144 --ny 6144 > gpurun_out/mall_6144_t4.log 2>&1
run > gpurun_out/mall_4096_default.log 2>&1
echo DONE
