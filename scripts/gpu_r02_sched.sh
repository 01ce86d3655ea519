# job-queue-scheduled Llama-3-8B run with auto:1 gang placement + the 1-GPU point of the scaling harness
cd $GRAFT_REPO_ROOT; source scripts/gpu_step.sh
mkdir -p gpurun_out
run_step r02s_scheduled 900 python -c "import json; from tensorhive_fixed_amd import benchmarks as b; print(json.dumps(b.scheduled_training(1, steps=8, auto=True)))"
tail -n 1 gpurun_out/r02s_scheduled.log
run_step r02s_scaling 600 python -m tensorhive_fixed_amd bench scaling --gpus 1
tail -n 1 gpurun_out/r02s_scaling.log
