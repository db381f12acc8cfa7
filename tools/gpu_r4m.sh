#!/bin/bash
# r4m: probe -- the (h+v)*R form in the per-launch kind-5 kernel (no guard)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4m}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "gpurun_out/${name}_$TAG.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run ab_4096 500 env TB_WARMUP=300 AB_ROUNDS=3 python -u tools/ab_env.py "" "CFD_PERSIST=0" "CFD_PERSIST=0,CFD_PROBE_LDS_SUMS=1"
run ab_c3 500 env AB_ROUNDS=2 AB_CMD="parity_one.py 4096 3" TB_WARMUP=100 python3 -u tools/ab_env.py "" "CFD_PROBE_LDS_SUMS=1"
run ab_slab4 400 env AB_CMD="tb_one.py 8192x2112@4096 5" TB_WARMUP=300 AB_ROUNDS=2 python3 -u tools/ab_env.py "" "CFD_PERSIST=0,CFD_PROBE_LDS_SUMS=1"
echo "=== done"
