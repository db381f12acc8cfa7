# Full GPU parity suite on the new defaults, then PMC traffic of the default
# march at 4096^2 and 8192^2 (dispatch-budgeted: 30 developing steps), then
# the bench under a kernel trace.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "=== $name $(date +%T)"; local t0=$(date +%s.%N)
  timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; local rc=$?
  echo "=== $name rc=$rc $(python3 -c "print(round($(date +%s.%N)-$t0,1))") s"; tail -3 gpurun_out/$name.log
  [ $rc -eq 0 ] || exit $rc; }
step pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
for N in 4096 8192; do
  A="--no-cpu-baseline --no-parity --no-control --develop 30 --warmup 0 --steps 2 --nx $N --ny $N"
  step pmc_fetch_$N 170 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_r2c_$N -o fetch --output-format csv -- python3 bench.py $A
  step pmc_write_$N 170 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_r2c_$N -o write --output-format csv -- python3 bench.py $A
  python3 tools/pmc_traffic.py gpurun_out/pmc_r2c_$N/fetch_counter_collection.csv gpurun_out/pmc_r2c_$N/write_counter_collection.csv --workload ${N}x${N} --command "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE (separate runs) -- python3 bench.py $A" -o gpurun_out/pmc_r2c_$N/pmc_traffic.json
done
step bench 600 python bench.py
step rocprof_stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-parity
echo DONE
