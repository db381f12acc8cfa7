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
  for pass in sq fetch write; do
    case $pass in
      sq) C="$CTRS";;
      fetch) C="FETCH_SIZE";;
      write) C="WRITE_SIZE";;
    esac
    CFD_TB_KIND=$K CFD_TEMPORAL=$T CFD_TB_ROWS=$R timeout -k 10 300 \
      rocprofv3 --pmc $C -d gpurun_out/pmc_$TAG -o ${name}_$pass --output-format csv \
      -- python3 tools/tb_one.py 4096 2 > gpurun_out/pmc_$TAG/${name}_$pass.log 2>&1
    rc=$?
    echo "rc=$rc"; tail -1 gpurun_out/pmc_$TAG/${name}_$pass.log
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
