#!/bin/bash
# Runs on the GPU box (via gpurun): GPU parity tests, smoke, bench, rocprof.
# Each GPU step has its own time limit; stop at the first failure / timeout.
#   TAG=<name>  PYTEST=0|1  TUNE=0|1  PROFILE=0|1  PMC=0|1  tools/gpu_check.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r2}
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
if [ "${PYTEST:-1}" = 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${TUNE:-0}" = 1 ]; then
  step tune 600 python tools/tune_tb.py 4096
fi
if [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  # the bench's main workload alone (its 8192^2 control launches the same
  # kernel name, so it gets its own trace: the stats then average one size each)
  step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --no-cpu-baseline --no-parity --no-control
  step rocprof_control 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o control --output-format csv -- python bench.py --no-cpu-baseline --no-parity --no-control --nx 8192 --ny 8192 --steps 10
fi
if [ "${PMC:-0}" = 1 ]; then
  # dispatch budget: 30 developing steps = ~1,000 dispatches (< 1 ms of
  # counter collection each, r2), one counter group per run
  export TMPDIR=/tmp
  step pmc_fetch 300 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_$TAG -o fetch --output-format csv -- python bench.py --no-cpu-baseline --no-parity --no-control --develop 30 --warmup 0 --steps 2
  step pmc_write 300 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_$TAG -o write --output-format csv -- python bench.py --no-cpu-baseline --no-parity --no-control --develop 30 --warmup 0 --steps 2
  step pmc_valu 300 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/pmc_$TAG -o valu --output-format csv -- python bench.py --no-cpu-baseline --no-parity --no-control --develop 30 --warmup 0 --steps 2
  python tools/pmc_valu.py gpurun_out/pmc_$TAG/valu_counter_collection.csv --workload 4096x4096 --command "python bench.py --no-cpu-baseline --no-parity --no-control --develop 30 --warmup 0 --steps 2" -o gpurun_out/pmc_$TAG/pmc_valu.json
  python tools/pmc_traffic.py gpurun_out/pmc_$TAG/fetch_counter_collection.csv gpurun_out/pmc_$TAG/write_counter_collection.csv --workload 4096x4096 --command "python bench.py --no-cpu-baseline --no-parity --no-control --develop 30 --warmup 0 --steps 2" -o gpurun_out/pmc_$TAG/pmc_traffic.json
fi
echo DONE
