#!/bin/bash
# GPU box: SQ counters for the Jacobi kernels of a few launch geometries.
# Usage: bash tools/pmc_tb.sh TAG "kind,T,R;kind,T,R"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
TAG=$1
CFGS=${2:-"1,4,24;1,4,32;3,8,24"}
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"}
mkdir -p gpurun_out/pmc_$TAG
IFS=';' read -ra LIST <<< "$CFGS"
for c in "${LIST[@]}"; do
  IFS=',' read -r K T R <<< "$c"
  name="k${K}_t${T}_r${R}"
  echo "=== $name $(date +%T)"
  CFD_TB_KIND=$K CFD_TEMPORAL=$T CFD_TB_ROWS=$R timeout -k 10 300 \
    rocprofv3 --pmc $CTRS -d gpurun_out/pmc_$TAG -o $name --output-format csv \
    -- python3 tools/tb_one.py 4096 2 > gpurun_out/pmc_$TAG/$name.log 2>&1
  rc=$?
  echo "rc=$rc"; tail -3 gpurun_out/pmc_$TAG/$name.log
  if [ $rc -ge 124 ]; then exit $rc; fi
done
