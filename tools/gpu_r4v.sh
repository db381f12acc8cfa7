#!/bin/bash
# r4v: kernel traces of the final tree's reference-default and C3 parity-mode steps
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
D=gpurun_out/prof_r4v
mkdir -p $D
run() {  # run <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$D/${name}.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -1 "$D/${name}.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run stats_refdef 300 rocprofv3 --kernel-trace --stats -d $D -o refdef --output-format csv -- python3 tools/refdef_one.py 10
run stats_parity 300 rocprofv3 --kernel-trace --stats -d $D -o parity --output-format csv -- python3 tools/parity_one.py 4096 2
echo "=== done"
