#!/bin/bash
# PMC passes over the chained vs per-launch march (tb_one 4096, 30 steps):
# issue / wait attribution and instruction-cache behaviour.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp TB_WARMUP=30
D=gpurun_out/pmc_${TAG:-chain}
mkdir -p $D
for CH in ${CHS:-0 1}; do
  for P in "A:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_INSTS_LDS" "B:SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_WAIT_INST_LDS SQ_INSTS_SMEM"; do
    name=${P%%:*}; ctrs=${P#*:}
    echo "=== chain=$CH pass $name"
    CFD_JACOBI_CHAIN=$CH timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-include-regex "k_jacobi_(lds|chain)" -d $D -o c${CH}_$name --output-format csv -- python3 tools/tb_one.py 4096 2 > $D/c${CH}_$name.log 2>&1
    rc=$?; echo "rc=$rc"; tail -1 $D/c${CH}_$name.log | cut -c1-300
    [ $rc -eq 0 ] || exit $rc
  done
done
