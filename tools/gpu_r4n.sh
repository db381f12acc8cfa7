#!/bin/bash
# r4n: per-launch march with the guarded SUMS chain as the single-domain
# default: full GPU suite, smoke, A/Bs
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4n}
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -3 "gpurun_out/${name}_$TAG.log" | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
}
run suite 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run ab_4096 500 env TB_WARMUP=300 AB_ROUNDS=3 python -u tools/ab_env.py "" "CFD_PERSIST=1" "CFD_JACOBI_SUMS=0"
run ab_c3 500 env AB_ROUNDS=2 AB_CMD="parity_one.py 4096 3" TB_WARMUP=100 python3 -u tools/ab_env.py "" "CFD_JACOBI_SUMS=0"
run ab_slab4 400 env AB_CMD="tb_one.py 8192x2112@4096 5" TB_WARMUP=300 AB_ROUNDS=2 python3 -u tools/ab_env.py "" "CFD_PERSIST=1"
echo "=== done"
