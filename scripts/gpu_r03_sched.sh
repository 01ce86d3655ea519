# round 3: the headline's queue-scheduled half -- Llama-3-8B launched by the job queue (auto:1), tokens/s from the task log
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out/r03
run_step r03/scheduled 900 python -m tensorhive_fixed_amd.cli bench scheduled
grep '^{' gpurun_out/r03/scheduled.log | cut -c1-700
