cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probes/valu_rate > gpurun_out/valu_rate.log 2>&1; echo "probe rc=$?"
cat gpurun_out/valu_rate.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "kernel_variants" --timeout 120 --timeout-method thread > gpurun_out/pytest_kv5.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_kv5.log
[ $rc -eq 0 ] || exit $rc
TB_WARMUP=400 TUNE_CONFIGS="4,8,24;5,8,24;5,8,16;5,8,20;5,8,32;5,4,24;5,6,24" timeout -k 10 500 python tools/tune_tb.py 4096 > gpurun_out/tune_r2b.log 2>&1; echo "tune rc=$?"; cat gpurun_out/tune_r2b.log
