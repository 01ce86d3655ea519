#!/usr/bin/env bash
# One gpurun session: build kernels, run GPU tests, short benches, optional rocprof.
# Every GPU step has its own time limit; a fault/abort/timeout (124,134,137,139) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if fatal $rc; then echo "FATAL rc=$rc in $name: stopping"; exit $rc; fi
  return 0
}
python -m tensorhive_fixed_amd.ops.build > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
for s in ${TH_STEPS:-tests bench}; do
  case $s in
    tests) step pytest_gpu 900 python -m pytest tests -m gpu -x -q ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_small) step bench_small 600 python bench.py --model llama3-1b-shape --steps 3 --warmup 1 ;;
    bench) step bench 900 python bench.py --steps ${TH_BENCH_STEPS:-5} --warmup 2 ;;
    kbench) step kbench 600 python scripts/bench_kernels.py ;;
    bench_plain) step bench_plain 900 env TH_DGRAD_NT=0 TH_WGRAD_NT=0 python bench.py --steps ${TH_BENCH_STEPS:-5} --warmup 2 ;;
    transpose_bw) step transpose_bw 300 python scripts/transpose_bw.py ;;
    layouts) step gemm_layouts 600 python scripts/gemm_layouts.py ;;
    flash) step flash_tests 600 python -m pytest tests/gpu/test_flash_attn_gpu.py -x -q ;;
    native) step native_tests 600 python -m pytest tests/gpu/test_native_gpu.py -x -q ;;
    doctor) step doctor 300 python -m tensorhive_fixed_amd doctor ;;
    daemon_bench) step daemon_bench 300 python -c "import json; from tensorhive_fixed_amd import benchmarks as b; print(json.dumps(b.poll_latency(1000))); print(json.dumps(b.launch_latency(5)))" ;;
    scheduled) step scheduled 900 python -c "import json; from tensorhive_fixed_amd import benchmarks as b; print(json.dumps(b.scheduled_training(1, steps=8)))" ;;
    prof) step prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 ;;
  esac
done
echo "== done"
