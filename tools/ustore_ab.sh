# predictor march u* store form A/B (dwordx4 at dword alignment vs 4 dwords)
export TMPDIR=/tmp
for v in us0 us1; do
  CFD_LIB=cfd-demo_amd/lib/variants/$v/libcfd_amd.so TB_WARMUP=200 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/us_$v -o run --output-format csv -- python3 tools/tb_one.py 4096 5 > gpurun_out/us_$v.log 2>&1 || exit 1
  grep -h predict_march gpurun_out/us_$v/run_kernel_stats.csv | cut -d, -f2-4 | tr -d '"'
done
CFD_LIB=cfd-demo_amd/lib/variants/us1/libcfd_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "fused or golden" 2>&1 | tail -1
