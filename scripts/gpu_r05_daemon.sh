# round 5: the headline's daemon halves on the final tree -- the queue-scheduled Llama-3-8B run (auto:1, the
# in-task HBM tool injected by th-run, tokens/s from the task log), the monitoring-overhead bench and the
# multi-tenant queue on the real node
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh; T=${TAG:-daemon3}
mkdir -p gpurun_out/r05/$T
run_step r05/$T/scheduled 900 python -m tensorhive_fixed_amd.cli bench scheduled
grep '^{' gpurun_out/r05/$T/scheduled.log | cut -c1-700
run_step r05/$T/overhead 600 python -m tensorhive_fixed_amd.cli bench overhead
grep '^{' gpurun_out/r05/$T/overhead.log | cut -c1-700
run_step r05/$T/mt_bench 500 python -m tensorhive_fixed_amd.cli bench multitenant --real
grep '^{' gpurun_out/r05/$T/mt_bench.log | cut -c1-900
