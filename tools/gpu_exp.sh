# Kind 5: boundary logic split (column patches per wave, row patches only in
# the slot groups that reach a boundary row) vs the previous build (head).
cd $GRAFT_REPO_ROOT
CFD_TB_KIND=5 CFD_TEMPORAL=8 TB_WARMUP=400 AB_ROUNDS=2 timeout -k 10 300 python tools/ab_variants.py head w11 > gpurun_out/ab_lds_edge.log 2>&1 || { tail -5 gpurun_out/ab_lds_edge.log; exit 1; }
cat gpurun_out/ab_lds_edge.log
CFD_LIB=$PWD/cfd-demo_amd/lib/variants/w11_stamp/libcfd_amd.so CFD_TB_KIND=5 CFD_TEMPORAL=8 timeout -k 10 120 python tools/lds_stamps.py 4096 > gpurun_out/stamps_w11.log 2>&1 || { tail -5 gpurun_out/stamps_w11.log; exit 1; }
cat gpurun_out/stamps_w11.log
CFD_LIB=$PWD/cfd-demo_amd/lib/variants/w11/libcfd_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_long.py > gpurun_out/pytest_w11.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_w11.log; exit $rc
