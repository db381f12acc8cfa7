#!/bin/bash
# GPU session runner.  Every step has its own time limit, steps are
# chained, and the script stops at the first failure (no retries).
#   TAG=r6a STAGES="suite smoke" tools/gpu_session.sh
# Stages: suite tests smoke bench stats pmc pmcsq ab abvar abslab refdef parity
# Outputs under gpurun_out/prof_$TAG.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r6}
D=gpurun_out/prof_$TAG
mkdir -p $D
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$D/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -3 "$D/$name.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
has() { [[ " $STAGES " == *" $1 "* ]]; }
B="python3 bench.py --no-cpu-baseline --no-parity --no-control --no-so --no-parity-mode --no-reference-default"
P="--develop 30 --warmup 0 --steps 2"

# the driver's GPU suite, exactly: unbuffered children as on its box
has suite && step suite 900 env PYTHONUNBUFFERED=1 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread
has tests && step tests 900 python -u -m pytest ${TESTS} -x -v -m gpu --timeout 400 --timeout-method thread
has smoke && step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
has bench && step bench_default 600 python3 bench.py
if has stats; then
  step stats_bench 300 rocprofv3 --kernel-trace --stats -d $D -o bench --output-format csv -- $B --steps 20 --warmup 5
  step stats_control 300 rocprofv3 --kernel-trace --stats -d $D -o control --output-format csv -- $B --nx 8192 --ny 8192 --steps 10
fi
if has parity; then
  step stats_parity 300 rocprofv3 --kernel-trace --stats -d $D -o parity --output-format csv -- python3 tools/parity_one.py 4096 2
fi
if has refdef; then
  step stats_refdef 300 rocprofv3 --kernel-trace --stats -d $D -o refdef --output-format csv -- python3 tools/refdef_one.py 10
fi
if has pmc; then
  for W in ${PMC_SIZES:-4096 8192}; do
    step pmc_fetch_$W 150 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D -o fetch_$W --output-format csv -- $B $P --nx $W --ny $W
    step pmc_write_$W 150 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D -o write_$W --output-format csv -- $B $P --nx $W --ny $W
    python3 tools/pmc_traffic.py $D/fetch_${W}_counter_collection.csv $D/write_${W}_counter_collection.csv --workload ${W}x${W} --command "$B $P --nx $W --ny $W" -o $D/pmc_traffic_${W}.json
    step pmc_valu_$W 150 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $D -o valu_$W --output-format csv -- $B $P --nx $W --ny $W
    python3 tools/pmc_valu.py $D/valu_${W}_counter_collection.csv --workload ${W}x${W} --command "$B $P --nx $W --ny $W" -o $D/pmc_valu_${W}.json
  done
fi
if has pmcsq; then
  # issue attribution of the dominant launch: LDS waits vs dependency stalls
  step pmc_sq_4096 150 timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $D -o sq_4096 --output-format csv -- $B $P --nx 4096 --ny 4096
fi
if has ab; then
  # AB_SETTINGS: space-separated env settings ("" = default), e.g. "'' CFD_X=1"
  step ab_${AB_NAME:-x} ${AB_SECS:-500} env AB_ROUNDS=${AB_ROUNDS:-3} AB_CMD="${AB_CMD:-tb_one.py 4096 5}" TB_WARMUP=${TB_WARMUP:-200} python3 -u tools/ab_env.py ${AB_SETTINGS}
fi
if has abvar; then
  # AB_VARIANTS: libraries built by tools/build_variants.sh (lib/variants/<name>)
  step abvar_${AB_NAME:-x} ${AB_SECS:-500} env AB_ROUNDS=${AB_ROUNDS:-3} AB_CMD="${AB_CMD:-tb_one.py 4096 5}" TB_WARMUP=${TB_WARMUP:-200} python3 -u tools/ab_variants.py ${AB_VARIANTS}
fi
if has abslab; then
  # persistent vs per-launch on the exact rank geometries (tb_one slab proxies
  # carry the owned rows + 2 x hg ghost rows; the pad is forced to the 24 KiB
  # the real slab gets from its OWNED rows -- the 16384 x 1088 proxy would
  # otherwise fall past the cache threshold and run unpadded)
  for shape in ${SLAB_SHAPES:-4096 8192x2112@4096 16384x1088@8192}; do
    step slab_$shape 420 env AB_CMD="tb_one.py $shape 5" TB_WARMUP=300 AB_ROUNDS=3 python3 -u tools/ab_env.py "CFD_PERSIST=0,CFD_LDS_PAD=24576" "CFD_PERSIST=1,CFD_LDS_PAD=24576"
  done
fi
echo "=== done"
