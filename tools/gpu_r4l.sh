#!/bin/bash
# r4l: resident solve (16 waves, finalize folded, tiles): spec tests, A/Bs, trace
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4l}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -5 "gpurun_out/${name}_$TAG.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run spec_tests 600 python -u -m pytest tests/test_gpu_spec.py -x -v -m gpu --timeout 300 --timeout-method thread
run ab_refdef 600 env AB_ROUNDS=2 AB_CMD="refdef_one.py 10" REFDEF_DEVELOP=100 python3 -u tools/ab_env.py "" "CFD_RESIDENT_ROWS=1" "CFD_RESIDENT_ROWS=4" "CFD_RESIDENT_T=4" "CFD_RESIDENT_TILE=16x112" "CFD_RESIDENT_TILE=16x112,CFD_RESIDENT_ROWS=4" "CFD_RESIDENT=0"
run ab_c2 400 env AB_ROUNDS=2 AB_CMD="parity_one.py 1024 5" TB_WARMUP=100 python3 -u tools/ab_env.py "" "CFD_RESIDENT=1" "CFD_RESIDENT=1,CFD_RESIDENT_ROWS=4"
run stats_refdef 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r4l -o refdef --output-format csv -- python3 tools/refdef_one.py 10
echo "=== done"
