cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
B="python3 bench.py --no-cpu-baseline --no-parity --no-control --no-so --no-parity-mode"
for r in 1 2; do
 for pad in default 0; do
  if [ $pad = default ]; then timeout -k 10 200 $B > gpurun_out/abb_${pad}_$r.log 2>&1 || exit 1
  else CFD_LDS_PAD=0 timeout -k 10 200 $B > gpurun_out/abb_${pad}_$r.log 2>&1 || exit 1; fi
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/abb_${pad}_$r.log') if l.startswith('{')][-1]); print('$pad', d['ms_per_step'], d['roofline']['avg_launch_us'])"
 done
done
timeout -k 10 300 python -u tools/ab_env.py "TB_WARMUP=400" "CFD_LDS_PAD=0,TB_WARMUP=400" > gpurun_out/ab_pad5.log 2>&1; tail -1 gpurun_out/ab_pad5.log
