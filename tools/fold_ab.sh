# Launch folds (step begin into the predictor march, step finalize into the
# finish's last workgroup): GPU suite, then per-step wall time with the folds
# on and off (CFD_CF_FOLD=0 keeps k_step_finalize; the begin fold has no knob).
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fold_pytest.log 2>&1; tail -2 gpurun_out/fold_pytest.log
for v in 1 0 1 0; do CFD_CF_FOLD=$v timeout -k 10 120 python tools/graph_ab.py 20 5 || exit 1; done
timeout -k 10 400 python bench.py --no-control > gpurun_out/fold_bench.log 2>&1; tail -c 300 gpurun_out/fold_bench.log
