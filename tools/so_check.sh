cd ${GRAFT_REPO_ROOT:-/root/repo} && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/so_parity.log 2>&1 || { tail -30 gpurun_out/so_parity.log; exit 1; }
tail -1 gpurun_out/so_parity.log
for v in 0 1; do
  CFD_PRED_VEC=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_so$v -o run --output-format csv -- python tools/so_step.py > gpurun_out/so_prof$v.log 2>&1 || exit 1
done
echo DONE
