#!/bin/bash
# Multigrid big-level smoother tile height (CFD_MG_TH_BIG) A/B: multigrid
# solve time per variant library (tools/build_variants.sh, VARIANT_TU=cfd_solvers),
# interleaved twice on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${VARIANTS:-th22 th30 th38 th46}; do
    echo -n "$v "
    CFD_LIB=cfd-demo_amd/lib/variants/$v/libcfd_amd.so timeout -k 10 120 python tools/bench_solvers.py --n 4096 --reps 10 --solvers 2 || exit 1
  done
done
