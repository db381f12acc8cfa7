#!/bin/bash
# Round-3 GPU session script (runs on the GPU box via gpurun).  Each GPU step
# has its own time limit; the script stops at the first failure or timeout.
#   TAG=<name> STEPS="new suite smoke bench prof" BENCH_ARGS=... tools/gpu_r3.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r3}
STEPS=${STEPS:-"suite smoke bench"}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -4 "gpurun_out/${TAG}_$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
for s in $STEPS; do
  case $s in
    new)   step new 900 $PYT -m gpu tests -k "${NEWK:-deadline or self_launch or developed}" ;;
    suite) step suite 1100 $PYT -m gpu tests ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    prof)
      export TMPDIR=/tmp
      step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run -- \
        python3 bench.py --no-cpu-baseline --no-control --no-parity --no-so --no-parity-mode ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== all done"
