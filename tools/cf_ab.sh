timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/cf_pytest.log 2>&1; tail -2 gpurun_out/cf_pytest.log
export TMPDIR=/tmp
for v in 0 1; do CFD_CF_MARCH=$v TB_WARMUP=200 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/cf_$v -o run --output-format csv -- python3 tools/tb_one.py 4096 5 > gpurun_out/cf_$v.log 2>&1 || exit 1; done
for v in 0 1; do CFD_CF_MARCH=$v timeout -k 10 120 python tools/graph_ab.py 20 5 || exit 1; done
