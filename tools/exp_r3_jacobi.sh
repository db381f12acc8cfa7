#!/bin/bash
# Round-3 Jacobi (kind 5) experiments on the GPU box: A/B of the variant
# libraries built by tools/build_variants.sh (VARIANT_TU=cfd_jacobi_lds8),
# then a segment-length sweep of the default library.  Every step has its own
# time limit; the script stops at the first failure.
#   VARIANTS="base d1 d3" TUNE_CONFIGS="5,8,-3;5,8,56" tools/exp_r3_jacobi.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-exp}
if [ -n "${VARIANTS:-}" ]; then
  AB_ROUNDS=${AB_ROUNDS:-3} timeout -k 10 600 python -u tools/ab_variants.py $VARIANTS \
    > gpurun_out/${TAG}_ab.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab.log; exit 1; }
  tail -3 gpurun_out/${TAG}_ab.log
fi
if [ -n "${TUNE_CONFIGS:-}" ]; then
  timeout -k 10 600 python -u tools/tune_tb.py 4096 > gpurun_out/${TAG}_tune.log 2>&1 || {
    tail -20 gpurun_out/${TAG}_tune.log; exit 1; }
  cat gpurun_out/${TAG}_tune.log
fi
echo "=== exp done"
