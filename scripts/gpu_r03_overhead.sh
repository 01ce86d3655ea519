# round 3: what the monitoring costs -- daemon CPU per sample, probe agent, tenant tokens/s with / without it
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/overhead 900 python -m tensorhive_fixed_amd.cli bench overhead
grep '^{' gpurun_out/r03/overhead.log
