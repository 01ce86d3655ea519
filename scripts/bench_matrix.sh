#!/usr/bin/env bash
# Run bench.py once per environment setting: bench_matrix.sh "A=1 B=2" "A=0" ...
# Each run has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m tensorhive_fixed_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
i=0
for setting in "$@"; do
  i=$((i+1))
  echo "== [$i] $setting ($(date +%T))"
  timeout -k 10 900 env $setting python bench.py --steps ${TH_BENCH_STEPS:-5} --warmup 2 > "gpurun_out/matrix_$i.log" 2>&1
  rc=$?
  echo "rc=$rc $setting"; grep '^{' "gpurun_out/matrix_$i.log" || tail -20 "gpurun_out/matrix_$i.log"
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
done
