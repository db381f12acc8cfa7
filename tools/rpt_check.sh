cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 2 4; do
  CFD_PRED_RPT=$r timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/rpt$r.log 2>&1 || { echo "FAIL rpt $r"; tail -30 gpurun_out/rpt$r.log; exit 1; }
  tail -1 gpurun_out/rpt$r.log
done
for rnd in 0 1; do
for r in 1 2 4; do
  CFD_PRED_RPT=$r timeout -k 10 120 python tools/tb_one.py 4096 5 >> gpurun_out/rpt_time.log 2>&1 || exit 1
done; done
for r in 1 2 4; do
  CFD_PRED_RPT=$r timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rpt$r -o run --output-format csv -- python tools/tb_one.py 4096 5 > /dev/null 2>&1 || exit 1
done
echo DONE
