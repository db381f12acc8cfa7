#!/bin/bash
# Predictor + divergence march (k_predict_march): GPU parity suite, then the
# per-kernel durations of the predictor kernels on the bench workload
# (first order: tile k_predict_div vs march at several segment lengths;
# second order: separate k_predict + k_divergence vs march).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${PYTEST:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pm_pytest.log 2>&1 || { tail -40 gpurun_out/pm_pytest.log; exit 1; }
  tail -2 gpurun_out/pm_pytest.log
fi
trace() {  # trace <tag> <script> [args]: kernel averages (us) of one traced run
  local tag=$1; shift
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pm_$tag -o run --output-format csv -- python3 "$@" > gpurun_out/pm_$tag.log 2>&1 || { tail -5 gpurun_out/pm_$tag.log; exit 1; }
  python3 - "$tag" <<'EOF'
import csv, glob, re, sys
tag = sys.argv[1]
for p in glob.glob(f"gpurun_out/pm_{tag}/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        n = r["Name"]
        if any(k in n for k in ("predict", "divergence", "correct_finish")):
            nm = re.search(r"k_\w+(<[^>]*>)?", n).group(0)
            print(f"{tag:>14} {nm:>44} calls {r['Calls']:>5} avg {float(r['AverageNs'])/1e3:8.2f} us")
EOF
}
for V in ${VARIANTS:-default}; do
  if [ "$V" = default ]; then L=""; else L=cfd-demo_amd/lib/variants/$V/libcfd_amd.so; fi
  CFD_LIB=$L TB_WARMUP=200 trace fo_$V tools/tb_one.py 4096 5
  CFD_LIB=$L trace so_$V tools/so_step.py
done
if [ "${SOLVERS:-0}" = 1 ]; then
  for v in 0 1; do
    CFD_SOR_FUSED=$v timeout -k 10 300 python tools/bench_solvers.py --n 4096 --iters 200 --reps 5 > gpurun_out/pm_solvers_sor$v.log 2>&1 || { tail -5 gpurun_out/pm_solvers_sor$v.log; exit 1; }
    echo "sor_fused=$v"; cat gpurun_out/pm_solvers_sor$v.log
  done
fi
echo DONE
