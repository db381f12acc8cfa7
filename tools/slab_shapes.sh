#!/bin/bash
# Per-sweep Jacobi time of the weak-scaling slab shapes on one GPU (verdict r3
# item 3): C3 4096^2, a C4 slab with its ghost rows (8192 x 2112) and a C5
# slab with its ghost rows (16384 x 1088), all at power-of-two spacing, with
# the LDS pad forced off / on and the default (keyed on owned rows since r4).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4}
for shape in 4096 8192x2112@4096 16384x1088@8192; do
  AB_CMD="tb_one.py $shape 5" TB_WARMUP=${TB_WARMUP:-300} timeout -k 10 400 python -u tools/ab_env.py \
    "" "CFD_LDS_PAD=0" "CFD_LDS_PAD=24576" > gpurun_out/slab_shape_${shape}_$TAG.log 2>&1
  rc=$?; tail -1 gpurun_out/slab_shape_${shape}_$TAG.log; [ $rc -eq 0 ] || exit $rc
done
