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
      step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline --no-control --no-parity --no-so --no-parity-mode ;;
    parity)
      # the reference's control flow (tolerance on) under the kernel tracer, C3 and C2
      export TMPDIR=/tmp
      step parity4096 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o parity4096 --output-format csv -- \
        python3 tools/parity_one.py 4096 3
      step parity1024 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o parity1024 --output-format csv -- \
        python3 tools/parity_one.py 1024 5 ;;
    cputable) step cputable 600 python3 tools/cpu_table.py --budget 15 ;;
    rehearse)
      # exactly as the driver invokes it (no external launcher); loopback puts
      # every rank on this box's one GPU (RCCL socket transport)
      step rehearse_n2 300 env CFD_BENCH_LOOPBACK=1 python3 bench.py --gpus 2
      step rehearse_n4 300 env CFD_BENCH_LOOPBACK=1 python3 bench.py --gpus 4
      # without loopback a 1-GPU box must refuse --gpus 2 (never an n_gpus 1 line)
      timeout -k 10 120 python3 bench.py --gpus 2 > gpurun_out/${TAG}_refuse_n2.log 2>&1
      echo "refuse_n2 rc=$?" | tee -a gpurun_out/${TAG}_refuse_n2.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== all done"
