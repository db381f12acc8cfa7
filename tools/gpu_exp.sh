# (1) the RCCL transport through the socket network on one GPU (two ranks,
# own NCCL_HOSTID each); (2) the r1 "PMC hang" command shape, timed: a full
# developed bench run (~12k dispatches) under one WRITE_SIZE pass.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "=== rccl_loopback $(date +%T)"
NCCL_DEBUG=WARN timeout -k 10 280 python3 tools/rccl_loopback.py --n 2 --steps 4 > gpurun_out/rccl_loopback.log 2>&1
rc=$?; echo "rc=$rc"; tail -20 gpurun_out/rccl_loopback.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "=== pmc_long $(date +%T)"
t0=$(date +%s)
timeout -s KILL 160 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_long -o write --output-format csv -- python3 bench.py --no-cpu-baseline --no-parity --no-control > gpurun_out/pmc_long.log 2>&1
rc=$?; echo "rc=$rc wall=$(( $(date +%s) - t0 )) s"; tail -2 gpurun_out/pmc_long.log | cut -c1-300
python3 - <<'PY'
import csv, collections
try:
    rows = list(csv.DictReader(open("gpurun_out/pmc_long/write_counter_collection.csv")))
    d = collections.Counter(r["Dispatch_Id"] for r in rows)
    ts = sorted(int(r["Start_Timestamp"]) for r in rows)
    print("dispatches", len(d), "span_s", (ts[-1] - ts[0]) / 1e9 if ts else None)
except Exception as e:
    print("no csv", e)
PY
