#!/bin/bash
# Round-3 profiling session on the GPU box (every step its own time limit;
# the script stops at the first failure).  Outputs under gpurun_out/prof_$TAG.
#   TAG=r3a tools/prof_r3.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r3}
D=gpurun_out/prof_$TAG
mkdir -p $D
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$D/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -3 "$D/$name.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python3 bench.py --no-cpu-baseline --no-parity --no-control --no-so --no-parity-mode"
P="--develop 30 --warmup 0 --steps 2"
if [ "${CALIB:-1}" = 1 ]; then
  step calib_fetch 120 timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $D -o calib_fetch --output-format csv -- ./tools/probes/fetch_calib
  step calib_write 120 timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $D -o calib_write --output-format csv -- ./tools/probes/fetch_calib
  BYTES=$(grep -o '"bytes_per_dispatch": [0-9]*' $D/calib_fetch.log | grep -o '[0-9]*$')
  python3 tools/pmc_calib.py $D/calib_fetch_counter_collection.csv $D/calib_write_counter_collection.csv --bytes $BYTES -o $D/fetch_calibration.json
fi
if [ "${STATS:-1}" = 1 ]; then
  step stats_bench 300 rocprofv3 --kernel-trace --stats -d $D -o bench --output-format csv -- $B
  step stats_control 300 rocprofv3 --kernel-trace --stats -d $D -o control --output-format csv -- $B --nx 8192 --ny 8192 --steps 10
  step stats_parity 300 rocprofv3 --kernel-trace --stats -d $D -o parity --output-format csv -- python3 tools/parity_one.py 4096 2
fi
if [ "${PMC:-1}" = 1 ]; then
  for W in 4096 8192; do
    step pmc_fetch_$W 150 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D -o fetch_$W --output-format csv -- $B $P --nx $W --ny $W
    step pmc_write_$W 150 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D -o write_$W --output-format csv -- $B $P --nx $W --ny $W
    python3 tools/pmc_traffic.py $D/fetch_${W}_counter_collection.csv $D/write_${W}_counter_collection.csv --workload ${W}x${W} --command "$B $P --nx $W --ny $W" -o $D/pmc_traffic_${W}.json
  done
  step pmc_valu 150 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $D -o valu --output-format csv -- $B $P
  python3 tools/pmc_valu.py $D/valu_counter_collection.csv --workload 4096x4096 --command "$B $P" -o $D/pmc_valu_4096.json
fi
if [ "${REHEARSE:-1}" = 1 ]; then
  # exactly as the driver invokes it (no external launcher); loopback puts
  # every rank on this box's one GPU (RCCL socket transport)
  step rehearse_n2 300 env CFD_BENCH_LOOPBACK=1 python3 bench.py --gpus 2
  step rehearse_n4 300 env CFD_BENCH_LOOPBACK=1 python3 bench.py --gpus 4
  # without loopback a 1-GPU box must refuse --gpus 2 (never an n_gpus 1 line)
  echo "=== refuse_n2"
  timeout -k 10 120 python3 bench.py --gpus 2 > $D/refuse_n2.log 2>&1
  echo "refuse_n2 rc=$?" | tee -a $D/refuse_n2.log
fi
echo "=== prof done"
