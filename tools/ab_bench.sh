#!/bin/bash
# A/B of environment settings on the bench's main leg, alternating, same box:
#   tools/ab_bench.sh "CFD_PERSIST=0" "CFD_PERSIST=1"      (ROUNDS=2)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline --no-parity --no-control --no-so --no-parity-mode"
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    tag=$(echo "$spec" | tr -c 'A-Za-z0-9' '_')
    env $(echo "$spec" | tr ',' ' ') timeout -k 10 200 $B > gpurun_out/abb_${tag}_$r.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abb_${tag}_$r.log') if l.startswith('{')][-1]); print('$spec', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],2))"
  done
done
