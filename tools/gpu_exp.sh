# Kernel trace of the bench workload (prio build = current source): launch
# durations and the gaps between consecutive Jacobi launches.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFD_LIB=$PWD/cfd-demo_amd/lib/variants/prio/libcfd_amd.so CFD_TB_KIND=5 CFD_TEMPORAL=8 TB_WARMUP=50 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_r2d -o kt -- python3 tools/tb_one.py 4096 3 > gpurun_out/kt_r2d.log 2>&1 || { tail -5 gpurun_out/kt_r2d.log; exit 1; }
tail -1 gpurun_out/kt_r2d.log
find gpurun_out/kt_r2d -name "*kernel_trace.csv"
