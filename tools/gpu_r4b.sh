set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
TAG=r4b tools/persist_check.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_sharded.py -k bench_geometry > gpurun_out/sharded_geom_r4b.log 2>&1; rc=$?; tail -5 gpurun_out/sharded_geom_r4b.log; [ $rc -eq 0 ] || exit $rc
TAG=r4b tools/slab_shapes.sh
