#!/bin/bash
# GPU box: SQ instruction/cycle counters of the Jacobi kernel only, one short
# run per launch geometry.  Usage: bash tools/pmc_sq.sh TAG "kind,T,R;..."
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp TB_WARMUP=${TB_WARMUP:-2}
TAG=$1
CFGS=${2:-"4,4,24;4,8,24"}
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY"}
mkdir -p gpurun_out/pmc_$TAG
IFS=';' read -ra LIST <<< "$CFGS"
for c in "${LIST[@]}"; do
  IFS=',' read -r K T R <<< "$c"
  name="k${K}_t${T}_r${R}"
  echo "=== $name $(date +%T)"
  CFD_TB_KIND=$K CFD_TEMPORAL=$T CFD_TB_ROWS=$R timeout -s KILL 150 \
    rocprofv3 --pmc $CTRS --kernel-include-regex "k_jacobi_(pipe|lds)" -d gpurun_out/pmc_$TAG \
    -o ${name} --output-format csv -- python3 tools/tb_one.py 4096 1 \
    > gpurun_out/pmc_$TAG/${name}.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -1 gpurun_out/pmc_$TAG/${name}.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
