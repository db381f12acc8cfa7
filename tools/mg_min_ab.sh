#!/bin/bash
# Smallest multigrid level smoothed by the row march (CFD_MG_MARCH_MIN, log2
# cells; smaller levels use the wave windows): 4096^2 solve times, interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for r in 1 2; do
  for v in ${MINS:-23 22 21 20}; do
    echo -n "min=$v "
    CFD_MG_MARCH_MIN=$v timeout -k 10 120 python tools/bench_solvers.py --n 4096 --reps 10 --solvers 2 || exit 1
  done
done
