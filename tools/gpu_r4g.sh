#!/bin/bash
# r4: full GPU suite + smoke, then A/Bs: persistent (SUMS form, acquire) and
# the parity-mode fusions.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4g}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/${name}_$TAG.log"
  [ $rc -eq 0 ] || { echo "ABORT after $name"; exit $rc; }
}
run persist_tests 600 python -u -m pytest tests/test_gpu_persist.py -x -v -m gpu --timeout 400 --timeout-method thread
run ab_persist 700 env TB_WARMUP=300 AB_ROUNDS=4 python -u tools/ab_env.py "" "CFD_JACOBI_SUMS=0" "CFD_PERSIST=0" "CFD_PERSIST_ACQ=0"
run suite 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run ab_parity 900 env AB_CMD="parity_one.py 4096 3" TB_WARMUP=100 python -u tools/ab_env.py "" "CFD_CORR_HEAD=0" "CFD_SPEC_FOLD=0" "CFD_CORR_HEAD=0,CFD_SPEC_FOLD=0"
