#!/bin/bash
# r4x: sanity of the final binary (smoke + spec/persist/parity tests)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4x.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_persist.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/tests_r4x.log 2>&1
rc=$?; tail -n 2 gpurun_out/smoke_r4x.log; tail -n 2 gpurun_out/tests_r4x.log; exit $rc
