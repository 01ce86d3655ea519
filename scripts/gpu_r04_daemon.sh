# round 4: the headline's daemon halves on the final tree -- the queue-scheduled Llama-3-8B run
# (auto:1, tokens/s from the task log) and the multi-tenant queue on the real node
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r04/daemon
run_step r04/daemon/scheduled 900 python -m tensorhive_fixed_amd.cli bench scheduled
grep '^{' gpurun_out/r04/daemon/scheduled.log | cut -c1-700
run_step r04/daemon/mt_bench 500 python -m tensorhive_fixed_amd.cli bench multitenant --real
grep '^{' gpurun_out/r04/daemon/mt_bench.log | cut -c1-700
