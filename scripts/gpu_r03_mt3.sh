# round 3: real-node multi-tenant harness, twice (device-freed wake + idle-claim re-checks), and its GPU test
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/mt_test 300 python -u -m pytest tests/gpu/test_multitenant_node_gpu.py -x -q --timeout 200 --timeout-method thread
tail -n 3 gpurun_out/r03/mt_test.log
run_step r03/mt_bench1 500 python -m tensorhive_fixed_amd.cli bench multitenant --real
tail -n 1 gpurun_out/r03/mt_bench1.log
run_step r03/mt_bench2 500 python -m tensorhive_fixed_amd.cli bench multitenant --real
tail -n 1 gpurun_out/r03/mt_bench2.log
