#!/bin/bash
# Multigrid row-march smoother (k_mg_smooth5m, CFD_MG_SMOOTH=2) vs the wave
# windows (k_mg_smooth5w, CFD_MG_SMOOTH=3): multigrid GPU parity tests, then
# 4096^2 solve times interleaved, then per-kernel stats of the march form.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "multigrid" --timeout 120 --timeout-method thread > gpurun_out/mgm_pytest.log 2>&1 || { tail -30 gpurun_out/mgm_pytest.log; exit 1; }
tail -1 gpurun_out/mgm_pytest.log
for r in 1 2; do
  for v in ${MODES:-3 2}; do
    echo -n "smooth=$v "
    CFD_MG_SMOOTH=$v timeout -k 10 120 python tools/bench_solvers.py --n 4096 --reps 10 --solvers 2 || exit 1
  done
done
CFD_MG_SMOOTH=2 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/mgm_prof -o run --output-format csv -- python3 tools/bench_solvers.py --n 4096 --reps 4 --solvers 2 > gpurun_out/mgm_prof.log 2>&1 || { tail -5 gpurun_out/mgm_prof.log; exit 1; }
python3 - <<'PY'
import csv, glob
for p in glob.glob("gpurun_out/mgm_prof/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "mg_" in r["Name"]:
            print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
