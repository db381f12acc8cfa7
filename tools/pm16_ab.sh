# First-order march: 8- vs 16-row segments (variant libraries), parity of the
# 16-row form, kernel times and step wall time.
export TMPDIR=/tmp
CFD_LIB=cfd-demo_amd/lib/variants/fo16/libcfd_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "fused or golden or full_size" > gpurun_out/pm16_pytest.log 2>&1; tail -1 gpurun_out/pm16_pytest.log
for v in fo8 fo16; do
  CFD_LIB=cfd-demo_amd/lib/variants/$v/libcfd_amd.so TB_WARMUP=200 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pm16_$v -o run --output-format csv -- python3 tools/tb_one.py 4096 5 > gpurun_out/pm16_$v.log 2>&1 || exit 1
  grep -h predict_march gpurun_out/pm16_$v/run_kernel_stats.csv | cut -d, -f2-4
done
for v in fo8 fo16 fo8 fo16; do CFD_LIB=cfd-demo_amd/lib/variants/$v/libcfd_amd.so timeout -k 10 120 python tools/graph_ab.py 20 5 || exit 1; done
