#!/bin/bash
# r4h: 8192^2 one-round persistent geometry check, reference-default kernel
# trace, slab-shape A/B, loopback rehearsals.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r4h}
D=gpurun_out/prof_$TAG
mkdir -p $D
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$D/${name}.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -2 "$D/${name}.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run persist_tests 400 python -u -m pytest tests/test_gpu_persist.py -x -q -m gpu --timeout 300 --timeout-method thread
run tb_8192 200 env TB_WARMUP=100 python3 tools/tb_one.py 8192 5
run stats_refdef 300 rocprofv3 --kernel-trace --stats -d $D -o refdef --output-format csv -- python3 tools/refdef_one.py 10
for shape in 4096 8192x2112@4096 16384x1088@8192; do
  run slab_shape_$shape 420 env AB_CMD="tb_one.py $shape 5" TB_WARMUP=300 python3 -u tools/ab_env.py "" "CFD_LDS_PAD=0" "CFD_PERSIST=0"
done
run rehearse_n2 400 env CFD_BENCH_LOOPBACK=1 python3 bench.py --gpus 2
run rehearse_n4 500 env CFD_BENCH_LOOPBACK=1 python3 bench.py --gpus 4
echo "=== done"
