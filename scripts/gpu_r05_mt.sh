# round 5: multi-tenant queue on the real node with task-exit events (hand-off from exit / from "done")
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
T=${TAG:-daemon}; mkdir -p gpurun_out/r05/$T
run_step r05/$T/mt_bench 500 python -m tensorhive_fixed_amd.cli bench multitenant --real
grep '^{' gpurun_out/r05/$T/mt_bench.log | cut -c1-900
