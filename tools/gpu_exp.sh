# Fused predictors + divergence (tile): parity, then timing vs unfused
# and per-kernel durations for 2 and 4 rows per tile.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sharded.py > gpurun_out/pytest_pd.log 2>&1 || { tail -30 gpurun_out/pytest_pd.log; exit 1; }
tail -2 gpurun_out/pytest_pd.log
for v in 0 1 0 1; do CFD_PRED_DIV=$v TB_WARMUP=400 timeout -k 10 120 python tools/tb_one.py 4096 10 | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print('pred_div=$v', round(d['ms_per_step'],4), round(d['us_per_sweep'],3), d['state_crc32'])" || exit 1; done
for R in 2 4; do
CFD_PRED_DIV_RPT=$R TB_WARMUP=20 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_pd$R -o kt -- python3 tools/tb_one.py 4096 3 > gpurun_out/kt_pd$R.log 2>&1 || { tail -5 gpurun_out/kt_pd$R.log; exit 1; }
done
echo traced
