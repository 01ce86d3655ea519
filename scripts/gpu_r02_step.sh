# step-level check of the current tree: default bench (3 runs) after the flash GPU tests
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
run_step r02s_bench1 400 python bench.py --steps 10 --warmup 3
run_step r02s_bench2 400 python bench.py --steps 10 --warmup 3
grep -h metric gpurun_out/r02s_bench1.log gpurun_out/r02s_bench2.log | python -c "import sys,json; [print(json.loads(l)['value'], json.loads(l)['ms_per_step']) for l in sys.stdin]"
