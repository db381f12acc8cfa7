# Solve finalize folded into the corrector finish (CFD_SOLVE_FIN_FOLD): GPU
# suite, then per-step wall time with the fold on and off.
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/fin_pytest.log 2>&1; tail -2 gpurun_out/fin_pytest.log
for v in 1 0 1 0; do CFD_SOLVE_FIN_FOLD=$v timeout -k 10 120 python tools/graph_ab.py 20 5 || exit 1; done
