#!/bin/bash
# Runs on the GPU box (via gpurun): GPU parity tests, smoke, bench, rocprof.
# Each GPU step has its own time limit; stop at the first timeout / signal.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${1:-r1}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
step pytest_gpu 900 python -m pytest tests -x -q -m gpu
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 10 --warmup 2
if [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
fi
if [ "${PMC:-0}" = 1 ]; then
  export TMPDIR=/tmp
  step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_$TAG -o fetch --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
  step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_$TAG -o write --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
fi
echo DONE
