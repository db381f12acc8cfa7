#!/bin/bash
# Round-4 profiling session on the GPU box (every step its own time limit; the
# script stops at the first failure).  Outputs under gpurun_out/prof_$TAG.
#   TAG=r4a tools/prof_r4.sh            (BENCH=1 STATS=1 PMC=1 SLABS=0 REHEARSE=0 by default)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r4}
D=gpurun_out/prof_$TAG
mkdir -p $D
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$D/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -2 "$D/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
B="python3 bench.py --no-cpu-baseline --no-parity --no-control --no-so --no-parity-mode --no-reference-default"
P="--develop 30 --warmup 0 --steps 2"
if [ "${SUITE:-0}" = 1 ]; then
  step suite 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread
  step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${BENCH:-1}" = 1 ]; then
  # the driver's command, unprofiled: the line whose kernel time the stats must agree with
  step bench_default 600 python3 bench.py
fi
if [ "${STATS:-1}" = 1 ]; then
  step stats_bench 300 rocprofv3 --kernel-trace --stats -d $D -o bench --output-format csv -- $B --steps 20 --warmup 5
  step stats_control 300 rocprofv3 --kernel-trace --stats -d $D -o control --output-format csv -- $B --nx 8192 --ny 8192 --steps 10
  step stats_parity 300 rocprofv3 --kernel-trace --stats -d $D -o parity --output-format csv -- python3 tools/parity_one.py 4096 2
fi
if [ "${PMC:-1}" = 1 ]; then
  for W in 4096 8192; do
    step pmc_fetch_$W 150 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D -o fetch_$W --output-format csv -- $B $P --nx $W --ny $W
    step pmc_write_$W 150 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D -o write_$W --output-format csv -- $B $P --nx $W --ny $W
    python3 tools/pmc_traffic.py $D/fetch_${W}_counter_collection.csv $D/write_${W}_counter_collection.csv --workload ${W}x${W} --command "$B $P --nx $W --ny $W" --persist-blocks 25 -o $D/pmc_traffic_${W}.json
    step pmc_valu_$W 150 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $D -o valu_$W --output-format csv -- $B $P --nx $W --ny $W
    python3 tools/pmc_valu.py $D/valu_${W}_counter_collection.csv --workload ${W}x${W} --command "$B $P --nx $W --ny $W" --persist-blocks 25 -o $D/pmc_valu_${W}.json
  done
  # the N=4 / N=8 rank slabs (8192 x 2048 and 16384 x 1024 owned rows) as
  # single-domain proxies with their 32 + 32 ghost rows, at the global grids'
  # power-of-two spacing: same kernel, same geometry (pad keyed on owned rows)
  export TB_WARMUP=30   # rocprofv3 runs the program itself (no env hop)
  # a rank slab runs the persistent launch between its exchanges: profile that
  export CFD_PERSIST=1
  for S in 8192x2112@4096:8192x2048 16384x1088@8192:16384x1024; do
    SH=${S%%:*}; WL=${S##*:}
    C="TB_WARMUP=30 python3 tools/tb_one.py $SH 2"
    step pmc_fetch_$WL 150 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D -o fetch_$WL --output-format csv -- python3 tools/tb_one.py $SH 2
    step pmc_write_$WL 150 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D -o write_$WL --output-format csv -- python3 tools/tb_one.py $SH 2
    python3 tools/pmc_traffic.py $D/fetch_${WL}_counter_collection.csv $D/write_${WL}_counter_collection.csv --workload $WL --command "$C" --persist-blocks 25 --note "single-domain proxy $SH of the rank slab (owned rows + 2 x 32 ghost rows)" -o $D/pmc_traffic_${WL}.json
    step pmc_valu_$WL 150 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $D -o valu_$WL --output-format csv -- python3 tools/tb_one.py $SH 2
    python3 tools/pmc_valu.py $D/valu_${WL}_counter_collection.csv --workload $WL --command "$C" --persist-blocks 25 --note "single-domain proxy $SH of the rank slab" -o $D/pmc_valu_${WL}.json
  done
  unset CFD_PERSIST TB_WARMUP
fi
if [ "${SLABS:-0}" = 1 ]; then
  for shape in 4096 8192x2112@4096 16384x1088@8192; do
    step slab_shape_$shape 420 env AB_CMD="tb_one.py $shape 5" TB_WARMUP=300 python3 -u tools/ab_env.py "" "CFD_LDS_PAD=0" "CFD_LDS_PAD=24576" "CFD_PERSIST=1"
  done
fi
if [ "${REHEARSE:-0}" = 1 ]; then
  # exactly as the driver invokes it (no external launcher); loopback puts
  # every rank on this box's one GPU (RCCL socket transport)
  step rehearse_n2 400 env CFD_BENCH_LOOPBACK=1 python3 bench.py --gpus 2
  step rehearse_n4 500 env CFD_BENCH_LOOPBACK=1 python3 bench.py --gpus 4
fi
echo "=== prof done"
