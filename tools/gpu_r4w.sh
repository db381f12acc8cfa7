#!/bin/bash
# r4w: two-level barrier in the resident solve
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4w}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "gpurun_out/${name}_$TAG.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run spec_tests 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_persist.py -x -q -m gpu --timeout 300 --timeout-method thread
run ab_refdef 500 env AB_ROUNDS=3 AB_CMD="refdef_one.py 10" REFDEF_DEVELOP=100 python3 -u tools/ab_env.py "" "CFD_RESIDENT_KEEP=0"
echo "=== done"
