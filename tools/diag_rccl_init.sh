cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cat > /tmp/dl.py <<'PY'
import os, sys, time
sys.path.insert(0, "cfd-demo_amd")
os.environ["NCCL_HOSTID"] = "cfd-lonely-rank0"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
os.environ.setdefault("NCCL_NET", "Socket")
import cfdamd
uid = cfdamd.rccl_unique_id()
print("uid ok", flush=True)
t0 = time.monotonic()
try:
    cfdamd.Model(cfdamd.cavity_grid(64), cfdamd.SimulationParams.cavity(100.0, 8), device=0, n_ranks=2, rank=0, unique_id=uid)
    print("CREATED", flush=True)
except cfdamd.CfdError as e:
    print("CODE", e.code, round(time.monotonic() - t0, 1), str(e)[:300], flush=True)
PY
CFD_RCCL_TIMEOUT_S=5 NCCL_DEBUG=INFO timeout -k 5 60 python -u /tmp/dl.py > gpurun_out/dl.log 2>&1; echo rc=$? >> gpurun_out/dl.log
tail -30 gpurun_out/dl.log
