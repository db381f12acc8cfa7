#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4e}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -4 "gpurun_out/${name}_$TAG.log"
  [ $rc -eq 0 ] || { echo "ABORT after $name"; exit $rc; }
}
P="python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu"
run persist_tests 900 $P tests/test_gpu_persist.py
run ab_persist 600 env TB_WARMUP=300 AB_ROUNDS=5 python -u tools/ab_env.py "" "CFD_PERSIST=0" "CFD_PERSIST_ACQ=0"
