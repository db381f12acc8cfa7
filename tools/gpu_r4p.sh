#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4p}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "gpurun_out/${name}_$TAG.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run tests 600 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_spec.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread
run ab_4096 500 env TB_WARMUP=300 AB_ROUNDS=4 python -u tools/ab_env.py "" "CFD_JACOBI_SUMS=0" "CFD_PERSIST=1"
run ab_c3 500 env AB_ROUNDS=2 AB_CMD="parity_one.py 4096 3" TB_WARMUP=100 python3 -u tools/ab_env.py "" "CFD_JACOBI_SUMS=0"
echo "=== done"
