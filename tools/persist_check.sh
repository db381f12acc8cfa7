#!/bin/bash
# Persistent-solve check on the GPU box: its bitwise tests, then an A/B of
# per-launch vs persistent (ticketed launch; with and without the agent acquire).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r4}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_persist.py \
  > gpurun_out/persist_tests_$TAG.log 2>&1
rc=$?; tail -25 gpurun_out/persist_tests_$TAG.log; [ $rc -eq 0 ] || exit $rc
TB_WARMUP=400 timeout -k 10 500 python -u tools/ab_env.py "CFD_PERSIST=0" "CFD_PERSIST=1" "CFD_PERSIST=1,CFD_PERSIST_ACQ=0" \
  > gpurun_out/ab_persist_$TAG.log 2>&1
rc=$?; cat gpurun_out/ab_persist_$TAG.log; exit $rc
