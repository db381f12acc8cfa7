#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
AB_ROUNDS=2 AB_CMD="refdef_one.py 10" REFDEF_DEVELOP=100 timeout -k 10 600 python3 -u tools/ab_env.py "" "CFD_SPEC=0" "CFD_TEMPORAL=4" "CFD_TEMPORAL=2" "CFD_GRAPH=1" "CFD_SPEC=0,CFD_GRAPH=1" > gpurun_out/ab_refdef_r4i.log 2>&1
rc=$?; cat gpurun_out/ab_refdef_r4i.log | cut -c1-300; exit $rc
